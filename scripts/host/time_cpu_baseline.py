"""(build container only) Time the imported reference Env.step and the
faithful-structure restatement oracle/torch_ref.py side by side on this host,
same configs and thread counts: validates that the CPU baseline bench.py
reports on the GPU box measures what the reference would (BASELINE.md §3:
within +-20%). Imports the reference unmodified from /root/reference with
bytecode writing off; never runs on the GPU box.

Run: PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python scripts/host/time_cpu_baseline.py
"""
import os
import sys
import time

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch  # noqa: E402

import make_golden as mg  # noqa: E402  (imports the reference)
from torch_ref import TorchRefEnv  # noqa: E402


def timed(step, acts, seconds):
    step(acts[0])
    n, t0 = 0, time.perf_counter()
    while True:
        step(acts[n % len(acts)])
        n += 1
        if time.perf_counter() - t0 > seconds:
            break
    return (time.perf_counter() - t0) / n


def main():
    secs = float(os.environ.get("SECONDS_PER_CASE", "4"))
    for th in (1, os.cpu_count()):
        torch.set_num_threads(th)
        for P, A, O in ((65536, 3, 3), (1024, 3, 8)):
            g = torch.Generator().manual_seed(99)
            acts = [torch.stack([(torch.rand(P, A, generator=g) - 0.5) * 0.5,
                                 torch.rand(P, A, generator=g) - 0.5], 2) for _ in range(4)]
            ref, _ = mg.ref_env(num_parallel=P, num_agents=A, num_obstacles=O)
            t_ref = timed(ref.step, acts, secs)
            port = TorchRefEnv(P, A, O, seed=7)
            t_port = timed(port.step, acts, secs)
            print(f"threads {th:3d} P{P} A{A} O{O}: reference {1e3 * t_ref:7.1f} ms/step, "
                  f"torch_ref {1e3 * t_port:7.1f} ms/step, ratio {t_port / t_ref:.2f}",
                  flush=True)


if __name__ == "__main__":
    main()
