"""The HIP kernel's acos over every fp32 in [-1, 1] (GPU box; generating script
for tests/golden/MANIFEST.json "acos_device").

The step kernels evaluate the bearing's acos (environment.py:286) with the
device library's acosf (acos_k, marl-nav_amd/csrc/device_math.h).
oracle/marlnav_oracle.c restates it op for op (acos_device), taking the
v_sqrt_f32 inside it from the measured table tests/golden/vsqrt_r_grid.npz
(scripts/probes/vsqrt_grid.py). This script runs the kernels' acos
(libmarlnav.so marlnav_debug_acos_range) and the library's acosf compiled
alone (scripts/probes/acos_lib.hip, the product's flags) over all
2 130 706 434 inputs in [-1, 1] and compares:

* kernel vs the oracle's restatement (must be equal on every input: this is
  what lets the GPU tests compare kernel and oracle bearings bit for bit);
* kernel, library acosf, glibc acosf and the correctly rounded acos vs MKL
  vsAcos (torch.acos on the host CPU: the reference's acos,
  tests/golden/libm_check.py) - how often each agrees with the reference.

usage (GPU box): python tests/golden/acos_dev_check.py [--quick] [--out FILE]
then fold FILE into MANIFEST.json with --merge FILE (host).
"""
import argparse
import ctypes
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import torch  # noqa: E402

import oracle as orc  # noqa: E402

ONE_BITS = 0x3F800000
CHUNK = 1 << 26


def ranges(step):
    out = []
    for base in (0, 0x80000000):
        first, last = base, base + ONE_BITS
        while first <= last:
            n = min(CHUNK, last - first + 1)
            out.append((first, n))
            first += n
    return out if step == 1 else out[::step]


def host_counts(first, n, dev, lib_acos):
    bits = (np.arange(n, dtype=np.uint64) + first).astype(np.uint32)
    x = bits.view(np.float32)
    restated = orc.acos_device_range(first, n)
    mkl = torch.acos(torch.from_numpy(x)).numpy()
    glibc = orc.acosf_range(first, n)
    cr = np.arccos(x.astype(np.float64)).astype(np.float32)
    eq = lambda a, b: int((a.view(np.uint32) == b.view(np.uint32)).sum())  # noqa: E731
    bad = np.flatnonzero(dev.view(np.uint32) != restated.view(np.uint32))
    return (np.array([n, eq(dev, restated), eq(dev, mkl), eq(glibc, mkl), eq(cr, mkl),
                      eq(dev, cr), eq(lib_acos, mkl), eq(lib_acos, dev), eq(lib_acos, cr)],
                     np.int64), [float(v) for v in x[bad[:4]]])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="every 8th chunk")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "acos_device.json"))
    ap.add_argument("--merge", help="(host) fold a result file into MANIFEST.json")
    a = ap.parse_args()
    if a.merge:
        with open(a.merge) as fh:
            res = json.load(fh)
        mpath = os.path.join(HERE, "MANIFEST.json")
        with open(mpath) as fh:
            man = json.load(fh)
        man["libm"]["acos_device"] = res
        with open(mpath, "w") as fh:
            json.dump(man, fh, indent=1, sort_keys=True)
            fh.write("\n")
        print("merged into", mpath)
        return
    import marlnav_amd as pkg
    lib = pkg.abi.load_library()   # the step kernels' acos (marlnav_debug_acos_range)
    libdev = ctypes.CDLL(os.path.join(ROOT, "scripts", "probes", "libacos.so"))
    libdev.acos_dev_range.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_void_p]
    torch.set_num_threads(1)
    t0 = time.time()
    tot = np.zeros(9, np.int64)
    ex = []
    buf = torch.empty(CHUNK, dtype=torch.float32, device="cuda")
    pending = []
    with ThreadPoolExecutor(12) as pool:
        for i, (first, n) in enumerate(ranges(8 if a.quick else 1)):
            assert lib.marlnav_debug_acos_range(first, n, buf.data_ptr(), None) == 0
            dev = buf[:n].cpu().numpy()   # synchronises
            assert libdev.acos_dev_range(first, n, buf.data_ptr(), None) == 0
            lib_acos = buf[:n].cpu().numpy()
            pending.append(pool.submit(host_counts, first, n, dev, lib_acos))
            if len(pending) >= 12:
                c, e = pending.pop(0).result()
                tot += c
                ex += e
            if i % 4 == 0:
                print(f"chunk {i} at {time.time() - t0:.0f} s", flush=True)
        for f in pending:
            c, e = f.result()
            tot += c
            ex += e
    n = int(tot[0])
    res = {
        "what": "the step kernels' bearing acos (acos_k: the device library's acosf) and "
                "that acosf compiled alone, over every fp32 in [-1, 1], against the oracle's "
                "restatement (acos_device with the measured v_sqrt_f32 table) and MKL; "
                "tests/golden/acos_dev_check.py on an MI355X",
        "inputs": n,
        "kernel_equals_oracle_acos_device": int(tot[1]),
        "kernel_not_equal_examples": ex[:8],
        "kernel_vs_mkl": tot[2] / n,
        "glibc_acosf_vs_mkl": tot[3] / n,
        "correctly_rounded_vs_mkl": tot[4] / n,
        "kernel_vs_correctly_rounded": tot[5] / n,
        "library_acosf_vs_mkl": tot[6] / n,
        "library_acosf_equals_kernel": int(tot[7]),
        "library_acosf_vs_correctly_rounded": tot[8] / n,
        "seconds": round(time.time() - t0, 1),
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))
    if not a.quick and int(tot[1]) != n:
        sys.exit(1)


if __name__ == "__main__":
    main()
