"""Host cost of the first timed steps of a fresh process (driver shape: 5
warm-up + 20 timed), under different pre-warming done before the warm-up."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import bench
import marlnav_amd as pkg

mode = sys.argv[1]
P = 65536
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
env = bench.make_env(pkg, P, 3, 3, dev, 0)
acts = bench.make_actions(P, 3, dev, 0)
if mode == "observe":
    for _ in range(64):
        env.observations()
elif mode == "torch":
    x = torch.zeros(16, device=dev)
    for _ in range(64):
        x.add_(1)
elif mode == "pool":
    outs = [env._take_outputs() for _ in range(4)]
    del outs
    for _ in range(64):
        env.observations()
torch.cuda.synchronize()
for i in range(5):
    env.step(acts[i % 64])
torch.cuda.synchronize()
ev0 = torch.cuda.Event(enable_timing=True)
ev1 = torch.cuda.Event(enable_timing=True)
ts = [time.perf_counter()]
if "ev" in sys.argv[2:]:
    ev0.record()
for i in range(20):
    env.step(acts[i % 64])
    ts.append(time.perf_counter())
if "ev" in sys.argv[2:]:
    ev1.record()
torch.cuda.synchronize()
te = time.perf_counter()
host = [round(1e6 * (b - a), 1) for a, b in zip(ts, ts[1:])]
print(f"{mode:8s} {sys.argv[2:]} wall/step {1e6 * (te - ts[0]) / 20:.2f} host {host}", flush=True)
