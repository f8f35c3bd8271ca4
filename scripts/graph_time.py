"""hipGraph-replay step time (as bench.py measures it) for alternative
libmarlnav builds at several configs, one process per call."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402


def main():
    import marlnav_amd as pkg
    libs = sys.argv[2:] or [pkg.abi.LIB_PATH]
    handles = [pkg.abi.load_library(p) for p in libs]
    for cfg in sys.argv[1].split(","):
        P, A, O = (int(x) for x in cfg.split("x"))
        dev = torch.device("cuda", 0)
        acts = bench.make_actions(P, A, dev, 0, n=8)
        for rep in range(int(os.environ.get("REPS", "2"))):
            for p, h in zip(libs, handles):
                args = pkg.default_args(num_parallel=P, num_agents=A, num_obstacles=O)
                params = pkg.set_env_params(args, dev)
                params.update(rng="native", seed=20251003, _lib=h)
                env = pkg.Env(params)
                for i in range(5):
                    env.step(acts[i % 8])
                avg, med = bench.kernel_time_us(env, acts)
                print(f"{cfg} {os.path.basename(p)} graph_us avg {avg:.2f} med {med:.2f}",
                      flush=True)
                del env


if __name__ == "__main__":
    main()
