"""Workload for PMC passes: N back-to-back Env.step at one config."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import marlnav_amd as pkg
P, A, O = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "65536x3x3").split("x"))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
params = pkg.set_env_params(pkg.default_args(num_parallel=P, num_agents=A, num_obstacles=O), "cuda")
params["rng"], params["seed"] = "native", 20251003
env = pkg.Env(params)
g = torch.Generator(device="cuda").manual_seed(1234)
acts = [torch.stack([torch.rand(P, A, generator=g, device="cuda") - 0.5,
                     torch.rand(P, A, generator=g, device="cuda") - 0.5], 2) for _ in range(8)]
for i in range(n):
    env.step(acts[i % 8])
torch.cuda.synchronize()
