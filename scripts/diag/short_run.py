"""Per-step host timings of the driver's short bench shape (5 warm-up + 20
timed steps), to see what the first steps after a synchronize cost."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import bench
import marlnav_amd as pkg

P = 65536
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
env = bench.make_env(pkg, P, 3, 3, dev, 0)
acts = bench.make_actions(P, 3, dev, 0)
for rep in range(3):
    for i in range(5):
        env.step(acts[i % 64])
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
    ts = [time.perf_counter()]
    evs[0].record()
    for i in range(20):
        env.step(acts[i % 64])
        evs[i + 1].record()
        ts.append(time.perf_counter())
    torch.cuda.synchronize()
    te = time.perf_counter()
    host = [round(1e6 * (b - a), 1) for a, b in zip(ts, ts[1:])]
    gpu = [round(1e3 * evs[i].elapsed_time(evs[i + 1]), 1) for i in range(20)]
    print("rep", rep, "wall/step %.2f" % (1e6 * (te - ts[0]) / 20))
    print("  host", host)
    print("  gpu ", gpu, flush=True)
