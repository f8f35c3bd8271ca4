"""Kernel micro-benchmark for the step kernel (GPU): per-launch HIP-event
durations with the host kept behind the GPU, for several configs, optionally
for alternative builds of libmarlnav.so (--lib a.so --lib b.so), interleaved
in one process (guide §5.4 rule 24)."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="65536x3x3,1024x3x8,4096x16x32,2097152x3x3")
    ap.add_argument("--lib", action="append", default=[])
    ap.add_argument("--launches", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import marlnav_amd as pkg
    libs = a.lib or [pkg.abi.LIB_PATH]
    handles = [pkg.abi.load_library(p) for p in libs]
    res = {}
    for cfg in a.configs.split(","):
        P, A, O = (int(x) for x in cfg.split("x"))
        params = pkg.set_env_params(pkg.default_args(num_parallel=P, num_agents=A,
                                                     num_obstacles=O), "cuda")
        params["rng"], params["seed"] = "native", 5
        env = pkg.Env(params)
        g = torch.Generator(device="cuda").manual_seed(1)
        acts = [torch.stack([torch.rand(P, A, generator=g, device="cuda") - 0.5,
                             torch.rand(P, A, generator=g, device="cuda") - 0.5], 2)
                for _ in range(8)]
        for _ in range(10):
            env.step(acts[0])
        times = {p: [] for p in libs}
        for _ in range(a.rounds):
            for p, h in zip(libs, handles):
                env._lib = h
                n = a.launches
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(n)]
                torch.cuda.synchronize()
                torch.cuda._sleep(int(80e6))
                for i in range(n):
                    ev[i][0].record()
                    env.step(acts[i % 8])
                    ev[i][1].record()
                torch.cuda.synchronize()
                times[p] += [s.elapsed_time(e) * 1e3 for s, e in ev]
        D = 2 + 2 * O + 2 * (A - 1)
        byt = P * ((28 * A + 8 * O + 13) + (20 * A + 4 * A * D + 11))
        for p in libs:
            t = sorted(times[p])
            med = statistics.median(t)
            res[f"{cfg}|{os.path.basename(p)}"] = {
                "median_us": round(med, 2), "min_us": round(t[0], 2),
                "mean_us": round(sum(t) / len(t), 2),
                "GBps_median": round(byt / (med * 1e-6) / 1e9, 1),
                "frac_8TBps": round(byt / (med * 1e-6) / 8e12, 3)}
        del env
    for k, v in res.items():
        print(k, json.dumps(v))


if __name__ == "__main__":
    main()
