"""Sub-phases of the pair-split kernel's workgroup-spread section (stamps
build, STAMPX slots 20..23: wave 0 after the row rewards, after the per-env
phase; every wave after the per-env barrier; after reinit_block) at one
config after WARM steps."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ["MARLNAV_LIB"] = os.path.join(ROOT, "marl-nav_amd", "lib", os.environ.get("STAMPS_LIB", "stamps.so"))
import numpy as np, torch  # noqa: E402
import marlnav_amd as pkg  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "4096x16x32"
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
for rep in range(3):
    buf.zero_()
    for i in range(8):
        env.step(acts[i % 8])
    torch.cuda.synchronize()
    raw = buf.view(nb, 24).cpu().numpy().astype(np.int64)
    raw = raw[raw[:, 0] > 0]
    us = lambda c: raw[:, c] * 10.0 / 1e3  # noqa: E731 (100 MHz ticks)
    s4, s5, s6 = us(8), us(10), us(12)
    w0 = raw[:, 20] > 0
    fin = raw[:, 19] > 0
    def med(x):
        return round(float(np.median(x)), 2) if x.size else None
    print(cfg, {"wave0 row rewards (S4->X0)": med((us(20) - s4)[w0]),
                "wave0 per-env (X0->X1)": med((us(21) - us(20))[w0]),
                "wave0 X1 -> barrier out (X2)": med((us(22) - us(21))[w0]),
                "nonfin: barrier out -> S5": med((s5 - us(22))[~fin & (raw[:, 22] > 0)]),
                "fin: barrier -> reinit done (X3)": med((us(23) - us(22))[fin & (raw[:, 23] > 0)]),
                "fin: reinit -> S5 (reobs)": med((s5 - us(23))[fin & (raw[:, 23] > 0)]),
                "S4->S5 fin / nonfin": (med((s5 - s4)[fin]), med((s5 - s4)[~fin])),
                "S5->S6 store": med(s6 - s5), "waves fin": int(fin.sum())})
