"""Per-phase timeline of the step kernel from the MARLNAV_STAMPS build
(marl-nav_amd/lib/stamps.so): block dispatch spread and phase durations."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["MARLNAV_LIB"] = os.path.join(ROOT, "marl-nav_amd", "lib",
                                         os.environ.get("STAMPS_LIB", "stamps.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import marlnav_amd as pkg
    cfgs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["65536x3x3"]
    names = ["staged", "moved", "observed", "env", "reobs", "stored", "drained"]
    for cfg in cfgs:
        P, A, O = (int(x) for x in cfg.split("x"))
        params = pkg.set_env_params(pkg.default_args(num_parallel=P, num_agents=A,
                                                     num_obstacles=O), "cuda")
        params["rng"], params["seed"] = "native", 5
        env = pkg.Env(params)
        lib = env._lib
        lib.marlnav_debug_stamps.argtypes = [ctypes.c_void_p]
        nb = P + 64  # >= waves of any step kernel (one env per wave at most)
        buf = torch.zeros(nb * 24, dtype=torch.int64, device="cuda")
        assert lib.marlnav_debug_stamps(buf.data_ptr()) == 0
        # bench.py's action stream (U(-0.5, 0.5) angle and acceleration)
        g = torch.Generator(device="cuda").manual_seed(1234)
        acts_l = [torch.stack([torch.rand(P, A, generator=g, device="cuda") - 0.5,
                               torch.rand(P, A, generator=g, device="cuda") - 0.5], 2)
                  for _ in range(8)]
        acts = acts_l[0]
        for i in range(int(os.environ.get("WARM", "5"))):
            env.step(acts_l[i % 8])
        torch.cuda.synchronize()
        res = []
        b2b = int(os.environ.get("B2B", "1"))
        for _ in range(5):
            for i in range(b2b):  # back-to-back launches: keep every XCD busy
                env.step(acts_l[i % 8])
            torch.cuda.synchronize()
            raw = buf.view(nb, 24).cpu().numpy().astype(np.int64)
            gidx = np.nonzero(raw[:, 0] > 0)[0]  # stamps slot = global wave index
            raw = raw[raw[:, 0] > 0]  # waves past the last tile record nothing
            fastw = (raw[:, 19] >> 8) & 1  # (split kernel: the wave took the short pair math)
            ownf = (raw[:, 19] >> 9) & 1   # (split kernel: the wave's own env finished)
            raw[:, 19] &= 0xff
            st = raw[:, :16].reshape(-1, 8, 2)
            entry = raw[:, 16] * 10.0 / 1e3
            rt = st[:, :, 0] * 10.0 / 1e3  # 100 MHz ticks -> us
            cy = st[:, :, 1]
            t0 = entry.min()
            ph = np.diff(rt, axis=1)
            clk = (cy[:, 7] - cy[:, 0]) / np.maximum(rt[:, 7] - rt[:, 0], 1e-3) / 1e3
            res.append({
                "span_us": round(float(rt[:, 7].max() - t0), 2),
                "entry_spread_us": round(float(entry.max() - t0), 2),
                "entry_to_t0_median_us": round(float(np.median(rt[:, 0] - entry)), 2),
                "entry_to_t0_p90_us": round(float(np.percentile(rt[:, 0] - entry, 90)), 2),
                "last_stored_us": round(float(rt[:, 6].max() - t0), 2),
                "phase_median_us": {n: round(float(np.median(ph[:, i])), 3)
                                    for i, n in enumerate(names)},
                "phase_p90_us": {n: round(float(np.percentile(ph[:, i], 90)), 3)
                                 for i, n in enumerate(names)},
                "block_total_median_us": round(float(np.median(rt[:, 7] - rt[:, 0])), 2),
                "clock_ghz_median": round(float(np.median(clk)), 2)})
        print(cfg, json.dumps(res[-1]))
        # entry time by XCC (dispatch placement)
        xcc = raw[:, 18] & 0xF
        e_rel = entry - entry.min()
        print(cfg, "entry_us by xcc (median, max):",
              {int(x): (round(float(np.median(e_rel[xcc == x])), 2),
                        round(float(e_rel[xcc == x].max()), 2)) for x in np.unique(xcc)})
        print(cfg, "entry percentiles us:", [round(float(np.percentile(e_rel, q)), 2)
                                             for q in (0, 10, 25, 50, 75, 90, 100)])
        print(cfg, "spans", [r["span_us"] for r in res])
        # SIMD load balance: waves per SIMD (HW_ID simd/cu/sh/se + XCC_ID) and
        # the end time of waves by their SIMD's wave count
        hw = raw[:, 17]
        key = ((xcc.astype(np.int64) << 16) | ((hw >> 13) & 7) << 12 | ((hw >> 12) & 1) << 8
               | ((hw >> 8) & 15) << 4 | ((hw >> 4) & 3))
        uk, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
        per_wave_cnt = cnt[inv]
        cu_key = key >> 4
        ucu, cu_cnt = np.unique(cu_key, return_counts=True)
        print(cfg, "simds used", len(uk), "waves/simd histogram",
              {int(k): int(v) for k, v in zip(*np.unique(cnt, return_counts=True))},
              "cus used", len(ucu), "waves/cu histogram",
              {int(k): int(v) for k, v in zip(*np.unique(cu_cnt, return_counts=True))})
        fin_all = rt[:, 7] - t0
        for c in np.unique(per_wave_cnt):
            m = per_wave_cnt == c
            print(cfg, f"waves on {int(c)}-wave SIMDs: n={int(m.sum())} end p50/p90/max us",
                  [round(float(np.percentile(fin_all[m], q)), 2) for q in (50, 90, 100)],
                  "chain p50", round(float(np.median(rt[m, 7] - entry[m])), 2))
        # the slowest 1% of waves: where their time went
        slow = fin_all >= np.percentile(fin_all, 99)
        print(cfg, "slowest 1% waves:", {"n": int(slow.sum()),
              "entry_us": round(float(np.median(entry[slow] - t0)), 2),
              "phase_median_us": {n: round(float(np.median(ph[slow, i])), 2)
                                  for i, n in enumerate(names)},
              "with_finished_envs": int((raw[slow, 19] > 0).sum())})
        # waves that re-observed finished envs vs the rest: do they set the end?
        reo = raw[:, 19] > 0  # tiles with a finished env (re-init + re-observe)
        if fastw.any():
            print(cfg, "short pair math: with finished envs", f"{fastw[reo].mean():.3f}",
                  "without", f"{fastw[~reo].mean():.3f}", flush=True)
        print(cfg, "clock GHz median: with finished envs", round(float(np.median(clk[reo])), 3),
              "without", round(float(np.median(clk[~reo])), 3),
              "| entry us median: with", round(float(np.median(entry[reo] - t0)), 2),
              "without", round(float(np.median(entry[~reo] - t0)), 2),
              "| observed-phase cycles median: with",
              int(np.median(cy[reo, 3] - cy[reo, 2])), "without", int(np.median(cy[~reo, 3] - cy[~reo, 2])),
              flush=True)
        if ownf.any():
            om = reo & (ownf == 1)
            nm = reo & (ownf == 0)
            print(cfg, "observed-phase cycles median in workgroups with finished envs: the finished env's wave",
                  int(np.median(cy[om, 3] - cy[om, 2])), f"(n={int(om.sum())})", "its other waves",
                  int(np.median(cy[nm, 3] - cy[nm, 2])) if nm.any() else None, f"(n={int(nm.sum())})",
                  flush=True)
        fin_t = rt[:, 7] - t0
        for name, m in (("with_reobs", reo), ("without", ~reo)):
            if m.any():
                print(cfg, name, {"waves": int(m.sum()),
                                  "chain_median_us": round(float(np.median(rt[m, 7] - entry[m])), 2),
                                  "end_p50_us": round(float(np.percentile(fin_t[m], 50)), 2),
                                  "end_p99_us": round(float(np.percentile(fin_t[m], 99)), 2),
                                  "end_max_us": round(float(fin_t[m].max()), 2),
                                  "phase_median_us": {n: round(float(np.median(ph[m, i])), 2)
                                                      for i, n in enumerate(names)}})
        # sub-phase stamps (STAMPX slots 20..23, realtime only) of waves in
        # tiles with finished envs: medians of consecutive differences, from
        # the phase-3 stamp (observed) through the X slots to the phase-5 stamp
        if reo.any():
            x = raw[reo][:, 20:24] * 10.0 / 1e3
            t3 = rt[reo][:, 3]
            t5 = rt[reo][:, 5]
            # XORDER: the order the X slots are reached in (default 0,1,2,3)
            xo = [int(v) for v in os.environ.get("XORDER", "0,1,2,3").split(",")]
            seq = [("observed", t3)] + [(f"x{k}", x[:, k]) for k in xo] + [("reobs_end", t5)]
            out = {}
            prev_name, prev = seq[0]
            for name, t in seq[1:]:
                m = (t > 0) & (prev > 0)
                if m.any():
                    out[f"{prev_name}->{name}"] = round(float(np.median(t[m] - prev[m])), 3)
                    prev_name, prev = name, t
            print(cfg, "with_reobs sub-phases (median us):", out)
            # the same per wave of the workgroup (WPB waves per workgroup:
            # A for the env-block kernel, 4 for the pair-split kernel)
            wpb = int(os.environ.get("WPB", str(A)))
            wid = gidx[reo] % wpb
            for w in range(wpb):
                m = wid == w
                if not m.any():
                    continue
                out = {}
                prev_name, prev = seq[0]
                for name, t in seq[1:]:
                    mm = m & (t > 0) & (prev > 0)
                    if mm.any():
                        out[f"{prev_name}->{name}"] = round(float(np.median(t[mm] - prev[mm])), 3)
                        prev_name, prev = name, t
                print(cfg, f"with_reobs wave {w} of {wpb}: env phase",
                      round(float(np.median(ph[reo][m, 3])), 3), "sub-phases", out,
                      "nfin histogram", {int(k): int(v) for k, v in
                                         zip(*np.unique(raw[reo][m, 19], return_counts=True))})
        # SUB=1 (substamps.so): the stage and observe sub-phases of every
        # agent wave (STAMPS_S slots 20..23: actions landed, sin/cos done,
        # spans landed; row computed)
        if os.environ.get("SUB") == "1":
            x = raw[:, 20:24] * 10.0 / 1e3
            ok = (x > 0).all(axis=1)
            if ok.any():
                seq = [("t0", rt[:, 0]), ("actions_landed", x[:, 0]), ("sincos_done", x[:, 1]),
                       ("spans_landed", x[:, 2]), ("stage_barrier", rt[:, 1]),
                       ("move_barrier", rt[:, 2]), ("row_computed", x[:, 3]),
                       ("observe_barrier", rt[:, 3])]
                for q in (50, 90):
                    out = {f"{a}->{b}": round(float(np.percentile((tb - ta)[ok], q)), 3)
                           for (a, ta), (b, tb) in zip(seq, seq[1:])}
                    print(cfg, f"stage/observe sub-phases (p{q} us, {int(ok.sum())} waves):", out)
                print(cfg, "entry->t0 median us", round(float(np.median((rt[:, 0] - entry)[ok])), 3))
            del env
            continue
        # wave 0's per-env phase (STAMPX 0..2 in wave 0: reward terms read,
        # outputs issued, list / counters done), every block
        w0 = (gidx % int(os.environ.get("WPB", str(A)))) == 0
        if w0.any():
            x = raw[w0][:, 20:23] * 10.0 / 1e3
            t3, t4 = rt[w0][:, 3], rt[w0][:, 4]
            ok = (x > 0).all(axis=1)
            if ok.any():
                seq = [("observed", t3), ("terms_read", x[:, 0]), ("outputs_issued", x[:, 1]),
                       ("counters_done", x[:, 2]), ("env_barrier", t4)]
                out = {f"{a}->{b}": round(float(np.median((tb - ta)[ok])), 3)
                       for (a, ta), (b, tb) in zip(seq, seq[1:])}
                print(cfg, "wave-0 per-env sub-phases (median us):", out)
        del env


if __name__ == "__main__":
    main()
