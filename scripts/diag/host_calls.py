"""Host time of each Env.step call in bench.py's timed-region shape (20 steps
right after a barrier-less torch.cuda.synchronize), per call index, median
over regions; and the same with the calls' HIP launch replaced by nothing
(the engine's host work alone cannot be isolated without a GPU, so the
comparison is against a plain torch op per call). GPU box."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
import marlnav_amd as pkg  # noqa: E402


def main():
    P = int(os.environ.get("P", "65536"))
    dev = torch.device("cuda", 0)
    env = bench.make_env(pkg, P, 3, 3, dev, 0)
    acts = bench.make_actions(P, 3, dev, 0)
    for i in range(50):
        env.step(acts[i % len(acts)])
    torch.cuda.synchronize()
    K, R = 20, int(os.environ.get("REGIONS", "30"))
    per = [[] for _ in range(K)]
    tot = []
    sync_t = []
    for r in range(R):
        for i in range(5):
            env.step(acts[i % len(acts)])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ts = [t0]
        for i in range(K):
            env.step(acts[i % len(acts)])
            ts.append(time.perf_counter())
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        for i in range(K):
            per[i].append((ts[i + 1] - ts[i]) * 1e6)
        tot.append((t2 - t0) * 1e6 / K)
        sync_t.append((t2 - ts[-1]) * 1e6)
    med = lambda v: sorted(v)[len(v) // 2]
    print("per-call host us (median over regions):", " ".join(f"{med(v):.1f}" for v in per))
    print(f"region us/step median {med(tot):.2f}; final synchronize wait median {med(sync_t):.1f} us; "
          f"host enqueue of 20 calls median {sum(med(v) for v in per):.1f} us")


if __name__ == "__main__":
    main()
