"""Where does a host-driven Env.step loop lose time? Host submission time vs
GPU timeline for several loop shapes (GPU box)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
import marlnav_amd as pkg

P = 65536
params = pkg.set_env_params(pkg.default_args(num_parallel=P), "cuda:0")
params["rng"], params["seed"] = "native", 20251003
env = pkg.Env(params)
g = torch.Generator(device="cuda:0").manual_seed(1234)
acts = [torch.stack([torch.rand(P, 3, generator=g, device="cuda:0") - 0.5,
                     torch.rand(P, 3, generator=g, device="cuda:0") - 0.5], 2).contiguous()
        for _ in range(64)]
zero = torch.zeros(P, 3, 2, device="cuda:0")


def run(name, fn, n, pre_sync=True):
    if pre_sync:
        torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter(); e0.record()
    for i in range(n):
        fn(i)
    t1 = time.perf_counter(); e1.record(); torch.cuda.synchronize(); t2 = time.perf_counter()
    print(f"{name:40s} n={n:4d} host_submit {1e6*(t1-t0)/n:6.2f} us/step  gpu {1e3*e0.elapsed_time(e1)/n:6.2f} us/step  wall {1e6*(t2-t0)/n:6.2f}", flush=True)


for rep in range(2):
    run("warm 50", lambda i: env.step(acts[i % 64]), 50)
    run("step rand acts x20", lambda i: env.step(acts[i % 64]), 20)
    run("step rand acts x500", lambda i: env.step(acts[i % 64]), 500)
    run("step zero acts x500", lambda i: env.step(zero), 500)
    run("step rand x500 no presync", lambda i: env.step(acts[i % 64]), 500, pre_sync=False)

# busy-spin the CPU before the timed region instead of a blocking sync
def spin_sync():
    ev = torch.cuda.Event()
    ev.record()
    while not ev.query():
        pass
for rep in range(2):
    run("warm", lambda i: env.step(acts[i % 64]), 50)
    spin_sync()
    run("after spin-sync: x20", lambda i: env.step(acts[i % 64]), 20, pre_sync=False)
