"""Graph-replay step-kernel time of the automatic kernel choice against each
forced family (marlnav_debug_force_family: 1 block, 2 split, 4 wave) over a
set of shapes; the same synthetic workload as bench.py (native triangle init,
U(-0.5, 0.5) actions). Usage: python scripts/diag/family_ab.py P,A,O [...]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import marlnav_amd as pkg  # noqa: E402

NAMES = {0: "auto", 1: "block", 2: "split", 4: "wave"}
shapes = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]] or [(16384, 3, 3)]
dev = "cuda"
for P, A, O in shapes:
    g = torch.Generator(device=dev).manual_seed(1234)
    acts = [(torch.rand(P, A, 2, generator=g, device=dev) - 0.5) for _ in range(8)]
    res = []
    for fam in tuple(int(f) for f in os.environ.get("FAMILIES", "0,1,2").split(",")):
        env = bench.make_env(pkg, P, A, O, dev, 0, seed=20251004)
        lib = env._lib
        prev = lib.marlnav_debug_force_family(fam)
        try:
            env.step(acts[0])
            torch.cuda.synchronize()
            ran = NAMES.get(lib.marlnav_debug_last_family(), "?")
            mean, med = bench.kernel_time_us(env, acts)
        finally:
            lib.marlnav_debug_force_family(prev)
        res.append(f"{NAMES[fam]}({ran}) {mean:.2f}/{med:.2f}")
        del env
        torch.cuda.empty_cache()
    print(f"{P}x{A}x{O}: " + "  ".join(res) + "  us mean/median", flush=True)
