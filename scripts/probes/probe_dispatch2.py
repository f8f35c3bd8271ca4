"""Per-XCC entry stagger of the step kernel's dispatch-only build, launched
through the C ABI with varying grid sizes, next to the plain probe kernel."""
import ctypes, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ["MARLNAV_LIB"] = os.path.join(ROOT, "marl-nav_amd", "lib", "stamps_dispatch.so")
import marlnav_amd as pkg
plib = ctypes.CDLL(os.path.join(ROOT, "scripts", "probes", "probe_lib.so"))
plib.probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]

def report(tag, raw):
    e = (raw[:, 0] - raw[:, 0].min()) * 0.01
    x = raw[:, 1] & 15
    print(tag, "spread %.2f" % e.max(), {int(k): round(float(e[x == k].min()), 2) for k in np.unique(x)},
          flush=True)

for P in (1024, 16384, 65536, 262144):
    params = pkg.set_env_params(pkg.default_args(num_parallel=P), "cuda")
    params["rng"], params["seed"] = "native", 5
    env = pkg.Env(params)
    lib = env._lib
    lib.marlnav_debug_stamps.argtypes = [ctypes.c_void_p]
    nb = env._counters.shape[1]
    buf = torch.zeros(nb * 24, dtype=torch.int64, device="cuda")
    lib.marlnav_debug_stamps(buf.data_ptr())
    acts = torch.zeros(P, 3, 2, device="cuda")
    for _ in range(6):
        buf.zero_()
        torch.cuda.synchronize()
        env.step(acts)
        torch.cuda.synchronize()
    raw = buf.view(nb, 24).cpu().numpy()
    raw = raw[raw[:, 0] > 0]
    report(f"step-kernel dispatch-only P={P} waves={len(raw)}", raw[:, [16, 18]])
    blocks = nb // 4
    t = torch.zeros(2 * blocks * 4, dtype=torch.int64, device="cuda")
    for _ in range(6):
        t.zero_()
        torch.cuda.synchronize()
        plib.probe_launch(t.data_ptr(), blocks, 256, 23000, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
    report(f"probe kernel blocks={blocks}", t.view(-1, 2).cpu().numpy())
