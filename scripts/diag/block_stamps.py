"""Sub-phases of the env-block kernel's fused re-init / re-observation pass
(stamps build, STAMPX slots 20..22 on waves 1..A-1: finished set known,
list visible, pass done) at one config after WARM steps."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ["MARLNAV_LIB"] = os.path.join(ROOT, "marl-nav_amd", "lib", os.environ.get("STAMPS_LIB", "stamps.so"))
import numpy as np, torch  # noqa: E402
import marlnav_amd as pkg  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "65536x3x3"
P, A, O = (int(x) for x in cfg.split("x"))
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
for i in range(int(os.environ.get("WARM", "150"))):
    env.step(acts[i % 8])
for rep in range(4):
    buf.zero_()  # one step per read-out: every stamp is from the same step
    env.step(acts[rep % 8])
    torch.cuda.synchronize()
    raw = buf.view(nb, 24).cpu().numpy().astype(np.int64)
    raw = raw[raw[:, 0] > 0]
    us = lambda c: raw[:, c] * 10.0 / 1e3  # noqa: E731
    s3, s4 = us(6), us(8)
    has = raw[:, 22] > 0
    w0 = (raw[:, 20] > 0) & ~has
    def med(x):
        return round(float(np.median(x)), 2) if x.size else None
    print(cfg, {"waves with pass": int(has.sum()),
                "S3 -> fin known (X0)": med((us(20) - s3)[has]),
                "X0 -> list visible (X1)": med((us(21) - us(20))[has]),
                "pass (X1 -> X2)": med((us(22) - us(21))[has]),
                "X2 -> barrier out (S4)": med((s4 - us(22))[has]),
                "S3->S4 with / without pass": (med((s4 - s3)[has]), med((s4 - s3)[w0]))})
