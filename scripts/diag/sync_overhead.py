"""Fixed overhead of bench.py's timed region (host clock minus GPU event
region) for 20-step loops: events recorded inside the region (bench.py), ev0
recorded before t0, no events; optional
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
KUS = bench.kernel_time_us(bench.make_env(pkg, P, A, O, dev, 0, seed=7), acts)[1]
print(f"graph-replay kernel time {KUS:.2f} us; overhead = host time of 20 steps - 20 x that")
for variant in ("device_sync", "ev0_before_t0", "no_events", "idle_sync_cost"):
    res = []
    for rep in range(15):
        torch.cuda.synchronize()
        if variant == "idle_sync_cost":
            t0 = time.perf_counter(); torch.cuda.synchronize(); res.append((time.perf_counter() - t0) * 1e6)
            continue
        if variant == "ev0_before_t0":
            e0.record()
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        if variant == "device_sync":
            e0.record()
        for i in range(20):
            env.step(acts[i % len(acts)])
        if variant != "no_events":
            e1.record()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e6
        res.append(dt - 20 * KUS)
    res.sort()
    print(f"{variant}: overhead us median {res[len(res)//2]:.1f} min {res[0]:.1f} max {res[-1]:.1f}", flush=True)
