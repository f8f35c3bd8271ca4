"""(GPU box) VERDICT r4 item 4: why the round-4 helper-wave build (a fourth
wave per env block at <= 256 blocks, commit f323b49) took 16384x3x3 from
5.62 to 8.22 us. Loads that revision's library (scripts/build_variant.sh
helper f323b49; helper_st = the same with -DMARLNAV_STAMPS=1) and toggles its
helper wave with its own testing hook (marlnav_debug_force_helper) between
runs: graph-replay step time (bench.kernel_time_us, steady mix) and, with
STAMPS=1, the per-phase wave stamps of scripts/kstamps.py.
With PMC_HELPER=h: 40 steps with the helper wave off/on, as a PMC workload.
usage: python scripts/diag/helper_diag.py lib.so [cfg]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
lib_path = os.path.abspath(sys.argv[1])
os.environ["MARLNAV_LIB"] = lib_path
cfg = sys.argv[2] if len(sys.argv) > 2 else "16384x3x3"
import torch  # noqa: E402
import bench  # noqa: E402
import marlnav_amd as pkg  # noqa: E402

lib = pkg.abi.load_library()
lib.marlnav_debug_force_helper.argtypes = [ctypes.c_int]
P, A, O = (int(x) for x in cfg.split("x"))
dev = torch.device("cuda", 0)
acts = bench.make_actions(P, A, dev, 0, n=16)
if os.environ.get("PMC_HELPER") is not None:  # a PMC workload (under rocprofv3 --pmc)
    lib.marlnav_debug_force_helper(int(os.environ["PMC_HELPER"]))
    params = pkg.set_env_params(pkg.default_args(num_parallel=P, num_agents=A, num_obstacles=O), dev)
    params.update(rng="native", seed=20251003)
    env = pkg.Env(params)
    for i in range(40):
        env.step(acts[i % 16])
    torch.cuda.synchronize()
    sys.exit(0)
for h in (0, 1, 0, 1):
    lib.marlnav_debug_force_helper(h)
    if os.environ.get("STAMPS") == "1":
        import kstamps
        print(f"helper={h} stamps", flush=True)
        sys.argv = [sys.argv[0], cfg]
        kstamps.main()
        continue
    args = pkg.default_args(num_parallel=P, num_agents=A, num_obstacles=O)
    params = pkg.set_env_params(args, dev)
    params.update(rng="native", seed=20251003)
    env = pkg.Env(params)
    bench.prewarm(env, acts, 0.2)
    env = pkg.Env(params)
    for i in range(150):
        env.step(acts[i % 16])
    env.allow_graph_capture = True
    print(f"{cfg} helper={h} steady graph replay us/step {bench.kernel_time_us(env, acts)[1]:.2f}",
          flush=True)
