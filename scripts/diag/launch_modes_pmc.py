"""PMC workload: the same Env.step launches as host stream launches (200)
and then as hipGraph replays (4 x 50), for per-dispatch counters
(rocprofv3 --pmc ... --kernel-trace): the dispatch order separates them."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402


def main():
    import marlnav_amd as pkg
    P, A, O = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "16384x3x3").split("x"))
    dev = torch.device("cuda", 0)
    acts = bench.make_actions(P, A, dev, 0, n=16)
    params = pkg.set_env_params(pkg.default_args(num_parallel=P, num_agents=A, num_obstacles=O), dev)
    params.update(rng="native", seed=20251003)
    env = pkg.Env(params)
    for i in range(300):
        env.step(acts[i % 16])
    torch.cuda.synchronize()
    for i in range(200):
        env.step(acts[i % 16])
    torch.cuda.synchronize()
    env.allow_graph_capture = True
    g = bench.capture_steps(env, acts, 50)
    torch.cuda.synchronize()
    for _ in range(4):
        g.replay()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
