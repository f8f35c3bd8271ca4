"""Per-tile phase timeline of the pipelined env-block kernel (MARLNAV_STAMPS
build with MARLNAV_BLOCK_PIPE=TP; STAMPS_LIB names it): the stamps slot of
env block blk is tile blk % TP of workgroup blk // TP, so the phases of each
tile position are reported apart, against the same kernel's first entry.
usage: STAMPS_LIB=stamps_pipe2.so TP=2 python scripts/diag/pipe_stamps.py 65536x3x3"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ["MARLNAV_LIB"] = os.path.join(ROOT, "marl-nav_amd", "lib",
                                         os.environ.get("STAMPS_LIB", "stamps.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

NAMES = ["staged", "moved", "observed", "env", "reobs", "stored", "drained"]


def main():
    import marlnav_amd as pkg
    tp = int(os.environ.get("TP", "2"))
    for cfg in (sys.argv[1] if len(sys.argv) > 1 else "65536x3x3").split(","):
        P, A, O = (int(x) for x in cfg.split("x"))
        params = pkg.set_env_params(pkg.default_args(num_parallel=P, num_agents=A,
                                                     num_obstacles=O), "cuda")
        params["rng"], params["seed"] = "native", 5
        env = pkg.Env(params)
        lib = env._lib
        lib.marlnav_debug_stamps.argtypes = [ctypes.c_void_p]
        nb = P + 64
        buf = torch.zeros(nb * 24, dtype=torch.int64, device="cuda")
        assert lib.marlnav_debug_stamps(buf.data_ptr()) == 0
        g = torch.Generator(device="cuda").manual_seed(1234)
        acts = [torch.stack([torch.rand(P, A, generator=g, device="cuda") - 0.5,
                             torch.rand(P, A, generator=g, device="cuda") - 0.5], 2)
                for _ in range(8)]
        for i in range(5):
            env.step(acts[i % 8])
        torch.cuda.synchronize()
        out = []
        for rep in range(3):
            env.step(acts[rep % 8])
            torch.cuda.synchronize()
            raw = buf.view(nb, 24).cpu().numpy().astype(np.int64)
            slots = np.nonzero(raw[:, 0] > 0)[0]
            raw = raw[slots]
            rt = raw[:, :16].reshape(-1, 8, 2)[:, :, 0] * 10.0 / 1e3
            entry = raw[:, 16] * 10.0 / 1e3
            t0 = entry.min()
            blk = slots // A
            tile = blk % tp
            res = {"span_us": round(float(rt[:, 7].max() - t0), 2)}
            for t in range(tp):
                m = tile == t
                ph = np.diff(rt[m], axis=1)
                res[f"tile{t}"] = {
                    "start_p50_us": round(float(np.median(rt[m, 0] - t0)), 2),
                    "end_p50_us": round(float(np.median(rt[m, 7] - t0)), 2),
                    "end_max_us": round(float((rt[m, 7] - t0).max()), 2),
                    "phase_p50_us": {n: round(float(np.median(ph[:, i])), 2)
                                     for i, n in enumerate(NAMES)}}
            out.append(res)
            print(cfg, json.dumps(res), flush=True)
        del env


if __name__ == "__main__":
    main()
