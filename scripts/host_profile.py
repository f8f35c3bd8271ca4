"""Host-side cost of Env.step and of its pieces (GPU box)."""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch

def t(fn, n=2000):
    for _ in range(100):
        fn()
    torch.cuda.synchronize()
    s = time.perf_counter()
    for _ in range(n):
        fn()
    e = time.perf_counter()
    torch.cuda.synchronize()
    return (e - s) / n * 1e6

import marlnav_amd as pkg
P = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
params = pkg.set_env_params(pkg.default_args(num_parallel=P), "cuda")
params["rng"], params["seed"] = "native", 5
env = pkg.Env(params)
acts = torch.zeros(P, 3, 2, device="cuda")
obs = torch.empty(P, 3, 12, device="cuda")
print("env.step            %.2f us" % t(lambda: env.step(acts)))
print("torch.empty x1      %.2f us" % t(lambda: torch.empty(P, 3, 12, device="cuda")))
print("torch.empty bool    %.2f us" % t(lambda: torch.empty(P, dtype=torch.bool, device="cuda")))
print("split6              %.2f us" % t(lambda: torch.split(obs, [1, 1, 3, 3, 2, 2], dim=2)))
print("current_stream      %.2f us" % t(lambda: torch.cuda.current_stream(env.device).cuda_stream))
print("raw stream          %.2f us" % t(lambda: torch._C._cuda_getCurrentRawStream(0)))
print("data_ptr            %.2f us" % t(lambda: obs.data_ptr()))
b = env._bufs
def setf():
    b.obs = obs.data_ptr()
print("struct field set    %.2f us" % t(setf))
lib = env._lib
d, p = ctypes.byref(env._dims), ctypes.byref(env._cparams)
bb = ctypes.byref(b)
print("ctypes byref        %.2f us" % t(lambda: ctypes.byref(env._dims)))
env._sync_params()
print("sync_params(clean)  %.2f us" % t(env._sync_params))
print("ctypes step call    %.2f us" % t(lambda: lib.marlnav_step(d, p, bb, 1, None)))
print("wrap_obs            %.2f us" % t(lambda: env._wrap_obs(obs)))
import cProfile, pstats
pr = cProfile.Profile()
pr.enable()
for _ in range(3000):
    env.step(acts)
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(20)
# the launch alone: ctypes call of marlnav_step with pre-set buffers
import numpy as np
print("is_capturing        %.2f us" % t(torch.cuda.is_current_stream_capturing))
print("take_outputs        %.2f us" % t(env._take_outputs))
o = env._out_pool[0]
print("set.free            %.2f us" % t(o.free))
o2 = env._take_outputs()
print("marlnav_step call   %.2f us" % t(lambda: lib.marlnav_step(env._dims_ref, env._cparams_ref, o2.bufs_ref, 1, torch._C._cuda_getCurrentRawStream(0))))
print("tiny torch op       %.2f us" % t(lambda: obs.add_(0)))
