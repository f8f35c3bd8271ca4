"""Same-box A/B of libmarlnav builds: hipGraph-replay step time (as bench.py
measures it) of a fresh Env (after 5 steps: few finished envs) and of one
stepped PRE steps further (episodes desynchronised by collisions: the steady
mix of finished envs per step), alternating the builds REPS times.
usage: python scripts/ab_steady.py 65536x3x3[,4096x16x32] lib1.so lib2.so ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402


def main():
    import marlnav_amd as pkg
    libs = sys.argv[2:] or [pkg.abi.LIB_PATH]
    handles = [pkg.abi.load_library(p) for p in libs]
    pre = int(os.environ.get("PRE", "150"))
    dev = torch.device("cuda", 0)
    for cfg in sys.argv[1].split(","):
        P, A, O = (int(x) for x in cfg.split("x"))
        acts = bench.make_actions(P, A, dev, 0, n=16)
        warm = None
        res = {p: {"fresh": [], "steady": []} for p in libs}
        for rep in range(int(os.environ.get("REPS", "3"))):
            for p, h in zip(libs, handles):
                args = pkg.default_args(num_parallel=P, num_agents=A, num_obstacles=O)
                params = pkg.set_env_params(args, dev)
                params.update(rng="native", seed=20251003, _lib=h)
                if os.path.basename(p) in os.environ.get("INPLACE", "").split(","):
                    params["states_double_buffer"] = False
                env = pkg.Env(params)
                if warm is None:  # clock ramp once per config
                    bench.prewarm(env, acts, 0.3)
                    warm = True
                    env = pkg.Env(params)
                for i in range(5):
                    env.step(acts[i % 16])
                res[p]["fresh"].append(bench.kernel_time_us(env, acts)[1])
                env.allow_graph_capture = False
                for i in range(pre):
                    env.step(acts[i % 16])
                res[p]["steady"].append(bench.kernel_time_us(env, acts)[1])
                del env
        for p in libs:
            f, s = sorted(res[p]["fresh"]), sorted(res[p]["steady"])
            print(f"{cfg} {os.path.basename(p):>16} fresh med {f[len(f) // 2]:.2f} "
                  f"{['%.2f' % x for x in res[p]['fresh']]}  steady med {s[len(s) // 2]:.2f} "
                  f"{['%.2f' % x for x in res[p]['steady']]}", flush=True)


if __name__ == "__main__":
    main()
