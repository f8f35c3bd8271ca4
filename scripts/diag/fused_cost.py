"""Graph-replay step-kernel time with the fused ObsNormalizer / ActionScaler
(MARLNAV_WRITE_OBS_NORM / MARLNAV_SCALE_ACTIONS) against the plain step, and
the unfused alternative (the normaliser as torch ops after the step), at
65536x3x3 (the MAPPO rollout shape of the headline config).
Usage: python scripts/diag/fused_cost.py [P]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import marlnav_amd as pkg  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
dev = "cuda"
args = pkg.default_args(num_parallel=P)
g = torch.Generator(device=dev).manual_seed(1234)
acts = [(torch.rand(P, 3, 2, generator=g, device=dev) - 0.5) for _ in range(8)]
for mode in ("plain", "norm", "scale", "norm+scale"):
    env = bench.make_env(pkg, P, 3, 3, dev, 0, seed=20251004)
    if "norm" in mode:
        env.attach_normalizer(pkg.ObsNormalizer(pkg.set_normalizer_params(args, dev)))
    if "scale" in mode:
        env.attach_action_scaler(pkg.ActionScaler(pkg.set_scaler_params(args, dev)))
    # the Python step loop as MAPPO drives it (host engine; timed like bench.py)
    import time
    for i in range(20):
        env.step(acts[i % 8])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(500):
        env.step(acts[i % 8])
    torch.cuda.synchronize()
    loop_us = (time.perf_counter() - t0) * 1e6 / 500
    mean, med = bench.kernel_time_us(env, acts)
    print(f"{P}x3x3 {mode}: graph-replay step {mean:.2f}/{med:.2f} us mean/median, "
          f"Python Env.step loop {loop_us:.2f} us/step", flush=True)
    del env
# unfused: the step, then the normaliser as torch ops on the packed obs
env = bench.make_env(pkg, P, 3, 3, dev, 0, seed=20251004)
nrm = pkg.ObsNormalizer(pkg.set_normalizer_params(args, dev))
env.allow_graph_capture = True
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for i in range(3):
        o, r, t, tr = env.step(acts[i])
        n = (o._packed - nrm.mean) / nrm.scale_tensor
torch.cuda.current_stream().wait_stream(side)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    for i in range(25):
        o, r, t, tr = env.step(acts[i % 8])
        n = (o._packed - nrm.mean) / nrm.scale_tensor
graph.replay()
torch.cuda.synchronize()
per = []
for _ in range(12):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    graph.replay()
    e.record()
    e.synchronize()
    per.append(s.elapsed_time(e) * 1e3 / 25)
per.sort()
print(f"{P}x3x3 step + torch normaliser: {sum(per) / len(per):.2f}/{per[len(per) // 2]:.2f} us", flush=True)
