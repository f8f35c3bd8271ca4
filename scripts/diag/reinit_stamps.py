"""Timeline inside the block kernel's fused re-init / re-observation pass
(waves 1..A-1 of blocks with finished envs), from a stamps build with extra
slots at wave + 8192 (0: call, 1: kernel args loaded, 2: env code read,
3: Philox done, 4: return) - a diagnostic build made by hand, not by the Makefile."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ["MARLNAV_LIB"] = os.path.join(ROOT, "marl-nav_amd", "lib", os.environ.get("STAMPS_LIB", "stamps_x.so"))
import numpy as np, torch  # noqa: E402
import marlnav_amd as pkg  # noqa: E402

P, A, O = 65536, 3, 3
params = pkg.set_env_params(pkg.default_args(num_parallel=P, num_agents=A, num_obstacles=O), "cuda")
params["rng"], params["seed"] = "native", 5
env = pkg.Env(params)
lib = env._lib
lib.marlnav_debug_stamps.argtypes = [ctypes.c_void_p]
nb = P + 64
buf = torch.zeros(nb * 24, dtype=torch.int64, device="cuda")
assert lib.marlnav_debug_stamps(buf.data_ptr()) == 0
g = torch.Generator(device="cuda").manual_seed(1234)
acts = [torch.stack([torch.rand(P, A, generator=g, device="cuda") - 0.5,
                     torch.rand(P, A, generator=g, device="cuda") - 0.5], 2) for _ in range(8)]
for i in range(12):
    env.step(acts[i % 8])
for rep in range(4):
    buf.zero_()
    env.step(acts[rep % 8])
    torch.cuda.synchronize()
    raw = buf.view(nb, 24).cpu().numpy().astype(np.int64)
    raw = raw[:3072]
    full = buf.view(nb, 24).cpu().numpy().astype(np.int64)
    ext = full[8192:8192 + len(full) - 8192][:len(raw)]
    m = (ext[:, 0] > 0) & (ext[:, 4] > 0)
    if not m.any():
        print("no re-init waves"); continue
    t = ext[m] * 10.0 / 1e3
    print(f"waves {int(m.sum())}")
    for name, a, b in (("call -> kernel args", 0, 1), ("args -> env code", 1, 2),
                       ("env code -> Philox done", 2, 3), ("Philox -> return", 3, 4),
                       ("whole call", 0, 4)):
        v = t[:, b] - t[:, a]
        v = v[(t[:, a] > 0) & (t[:, b] > 0)]
        if len(v):
            print(f"  {name}: median {np.median(v):.2f} p90 {np.percentile(v, 90):.2f} us (n={len(v)})")
