"""Round 6: the round trip of the one returning atomic a
cross-workgroup finished-env work list would cost each split-kernel workgroup
after its stores (MARLNAV_CLAIM_PROBE stamps build, slot 23 of wave 0 of each
workgroup), and when those workgroups end relative to the kernel's last wave.
The probe's code is in git history at a9bbeb6 (removed from the sources):
  scripts/build_variant.sh stclaim a9bbeb6 -DMARLNAV_CLAIM_PROBE=1 -DMARLNAV_STAMPS=1
usage: STAMPS_LIB=stclaim.so python scripts/diag/claim_rtt.py 4096x16x32"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ["MARLNAV_LIB"] = os.path.join(ROOT, "marl-nav_amd", "lib",
                                         os.environ.get("STAMPS_LIB", "stclaim.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import marlnav_amd as pkg
    for cfg in sys.argv[1].split(","):
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
        for i in range(int(os.environ.get("WARM", "150"))):
            env.step(acts[i % 8])
        rtts, ends, owner_ends, kend = [], [], [], []
        for rep in range(5):
            for i in range(8):
                env.step(acts[i % 8])
            torch.cuda.synchronize()
            raw = buf.view(nb, 24).cpu().numpy().astype(np.int64)
            gidx = np.nonzero(raw[:, 0] > 0)[0]
            raw = raw[raw[:, 0] > 0]
            w0 = gidx % 4 == 0
            t0 = raw[:, 16].min()
            end = (raw[:, 14] - t0) * 10.0 / 1e3  # STAMP(7): the wave's last stamp
            nfin = raw[:, 19] & 0xff
            rtts.append(raw[w0, 23] * 10.0 / 1e3)
            ends.append(end[w0 & (nfin == 0)])
            owner_ends.append(end[w0 & (nfin > 0)])
            kend.append(end.max())
        r = np.concatenate(rtts)
        e, oe = np.concatenate(ends), np.concatenate(owner_ends)
        q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (10, 50, 90, 99, 100)]
        print(cfg, "claim round trip us p10/50/90/99/max", q(r))
        print(cfg, "end of workgroups without finished envs us p10/50/90/99/max", q(e))
        print(cfg, "end of workgroups with finished envs us p10/50/90/99/max", q(oe),
              "kernel span us", [round(float(x), 2) for x in kend])


if __name__ == "__main__":
    main()
