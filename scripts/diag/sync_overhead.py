"""Fixed overhead of bench.py's timed region (host clock minus GPU event
region) for 20-step loops under several synchronisation variants; optional
hipDeviceScheduleSpin (argv[1] == 'spin', set before torch touches the GPU)."""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
if len(sys.argv) > 1 and sys.argv[1] == "spin":
    hip = ctypes.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags(spin) ->", hip.hipSetDeviceFlags(ctypes.c_uint(1)))
import torch  # noqa: E402
import bench  # noqa: E402
import marlnav_amd as pkg  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
P, A, O = 65536, 3, 3
env = bench.make_env(pkg, P, A, O, dev, 0)
acts = bench.make_actions(P, A, dev, 0)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); e1.record(); e1.synchronize()
for i in range(5):
    env.step(acts[i % len(acts)])
torch.cuda.synchronize()
for variant in ("device_sync", "event_then_device", "query_spin_then_device", "idle_sync_cost"):
    res = []
    for rep in range(15):
        torch.cuda.synchronize()
        if variant == "idle_sync_cost":
            t0 = time.perf_counter(); torch.cuda.synchronize(); res.append((time.perf_counter() - t0) * 1e6)
            continue
        t0 = time.perf_counter()
        e0.record()
        for i in range(20):
            env.step(acts[i % len(acts)])
        e1.record()
        if variant == "event_then_device":
            e1.synchronize()
        if variant == "query_spin_then_device":
            while not e1.query():
                pass
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e6
        reg = e0.elapsed_time(e1) * 1e3
        res.append(dt - reg)
    res.sort()
    print(f"{variant}: overhead us median {res[len(res)//2]:.1f} min {res[0]:.1f} max {res[-1]:.1f}", flush=True)
