"""Per-step GPU time of the same Env.step launches issued three ways, one
process, one box: (a) a host Python loop of K steps behind a device spin
(stream launches, the queue never empties), HIP events around the K steps;
(a') the same on a created stream; (b) a hipGraph of K captured steps replayed once (graph launches, one
replay boundary), HIP events around it; (c) the bench's host-clock region
(synchronize, K steps, synchronize). usage: python scripts/diag/launch_modes.py [65536x3x3] [K]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402


def main():
    import marlnav_amd as pkg
    P, A, O = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "65536x3x3").split("x"))
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    dev = torch.device("cuda", 0)
    acts = bench.make_actions(P, A, dev, 0, n=16)
    params = pkg.set_env_params(pkg.default_args(num_parallel=P, num_agents=A, num_obstacles=O), dev)
    params.update(rng="native", seed=20251003)
    env = pkg.Env(params)
    fam = int(os.environ.get("MARLNAV_FORCE_FAMILY", "0"))  # (include/marlnav.h MARLNAV_FAMILY_*)
    if fam:
        assert env._lib.marlnav_debug_force_family(fam) == 0
    bench.prewarm(pkg.Env(params), acts, 0.3)
    for i in range(300):  # the steady mix of finished envs
        env.step(acts[i % 16])
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {"stream": [], "side": [], "graph": [], "host20": []}
    side = torch.cuda.Stream()
    g = None
    for rep in range(5):
        torch.cuda._sleep(bench.SPIN_CYCLES)
        s.record()
        for i in range(K):
            env.step(acts[i % 16])
        e.record()
        e.synchronize()
        res["stream"].append(s.elapsed_time(e) * 1e3 / K)
        torch.cuda.synchronize()
        with torch.cuda.stream(side):  # the same on a created (non-default) stream
            torch.cuda._sleep(bench.SPIN_CYCLES)
            s.record()
            for i in range(K):
                env.step(acts[i % 16])
            e.record()
        e.synchronize()
        res["side"].append(s.elapsed_time(e) * 1e3 / K)
        torch.cuda.synchronize()
        if g is None:
            env.allow_graph_capture = True
            g = bench.capture_steps(env, acts, K)
            env.allow_graph_capture = False
        torch.cuda.synchronize()
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        res["graph"].append(s.elapsed_time(e) * 1e3 / K)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(20):
            env.step(acts[i % 16])
        torch.cuda.synchronize()
        res["host20"].append((time.perf_counter() - t0) * 1e6 / 20)
    for k, v in res.items():
        v = sorted(v)
        print(f"{P}x{A}x{O} K={K} {k:7s} us/step median {v[len(v) // 2]:.3f} {['%.2f' % x for x in v]}",
              flush=True)


if __name__ == "__main__":
    main()
