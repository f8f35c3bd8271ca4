"""Which libm the reference's CPU path evaluates, and which fp32 sin/cos
agrees with it most often (build container only; writes the "libm" entry of
tests/golden/MANIFEST.json).

The reference turns every heading with torch.sin / torch.cos
(environment.py:131-137, under vmap) and measures every bearing with
torch.acos (:286). In this torch build those CPU kernels are MKL VML:

1. identity: torch.sin/cos/acos equal vsSin/vsCos/vsAcos called through
   ctypes from libtorch_cpu.so, on random and structured fp32 inputs;
2. sweep: every fp32 angle in [-pi, pi] (the clamped action range,
   environment.py:115), ~2.16e9 values: how often MKL's sin and cos equal
   (i) the shipped oracle_sincos / kernel sincos_k (fp64 evaluation rounded
   once to fp32) and (ii) the round-2 fp32 Cephes sequence; and whether the
   shipped one is correctly rounded everywhere (numpy fp64 sin/cos rounded to
   fp32, disagreements adjudicated with long double sinl/cosl);
3. acos: every fp32 in [-1, 1]: MKL vsAcos against glibc acosf (the C
   oracle's) and against the correctly rounded acos.

Run: python tests/golden/libm_check.py [--quick]  (--quick: a 1/64 sample of
the sweeps, not recorded). About 2-4 minutes on 8 cores.
"""
import argparse
import ctypes
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
import oracle as orc  # noqa: E402

PI_BITS = int(np.float32(np.pi).view(np.uint32))    # 0x40490fdb, pi rounded up
ONE_BITS = int(np.float32(1.0).view(np.uint32))
CHUNK = 1 << 22


def vml():
    """vsSin / vsCos / vsAcos from the libtorch_cpu.so torch itself loaded."""
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "libtorch_cpu.so")
    lib = ctypes.CDLL(path)
    fns = {}
    for name in ("vsSin", "vsCos", "vsAcos"):
        f = getattr(lib, name)
        f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        f.restype = None
        fns[name] = f
    mode = None
    if hasattr(lib, "vmlGetMode"):
        lib.vmlGetMode.restype = ctypes.c_uint
        mode = int(lib.vmlGetMode())
    return fns, mode, path


def call_vml(f, x):
    x = np.ascontiguousarray(x, np.float32)
    y = np.empty_like(x)
    f(x.size, x.ctypes.data, y.ctypes.data)
    return y


def identity_check(fns):
    g = np.random.default_rng(7)
    xs = {
        "uniform[-pi,pi]": g.uniform(-np.pi, np.pi, 1 << 20).astype(np.float32),
        "uniform[-1e-3,1e-3]": g.uniform(-1e-3, 1e-3, 1 << 18).astype(np.float32),
        "uniform[-1,1]": g.uniform(-1, 1, 1 << 20).astype(np.float32),
        "near+-1": (1 - g.uniform(0, 1e-4, 1 << 18) * g.choice([-1, 1], 1 << 18)).astype(np.float32)
                   * g.choice([-1, 1], 1 << 18).astype(np.float32),
    }
    out = {}
    for name, x in xs.items():
        t = torch.from_numpy(x)
        r = {}
        for fn, tf in (("vsSin", torch.sin), ("vsCos", torch.cos), ("vsAcos", torch.acos)):
            a = call_vml(fns[fn], x)
            b = tf(t).numpy()
            r[fn] = float(np.mean((a.view(np.uint32) == b.view(np.uint32))
                                  | (np.isnan(a) & np.isnan(b))))
        out[name] = r
    # a (P, A) tensor like the reference's clamped action angles under vmap
    ang = torch.clamp(torch.from_numpy(g.uniform(-4, 4, (4096, 3)).astype(np.float32)),
                      -np.pi, np.pi)
    vm = torch.vmap(torch.vmap(lambda a: torch.stack([torch.cos(a), torch.sin(a)])))(ang)
    x = ang.numpy().ravel()
    out["vmap(vmap) as in _rotate"] = {
        "vsCos": float(np.mean(call_vml(fns["vsCos"], x) == vm[..., 0].numpy().ravel())),
        "vsSin": float(np.mean(call_vml(fns["vsSin"], x) == vm[..., 1].numpy().ravel())),
    }
    return out


def cr_from_f64(f64vals):
    return f64vals.astype(np.float32)


def sweep_chunk(first, n, step):
    """Counts over bit patterns first, first+step, ... (step > 1 only in --quick)."""
    s_new, c_new = orc.sincos_range(first, n, 0)
    s_old, c_old = orc.sincos_range(first, n, 1)
    bits = (np.arange(n, dtype=np.uint64) + first).astype(np.uint32)
    th = bits.view(np.float32)
    if step > 1:
        sel = slice(None, None, step)
        th, s_new, c_new, s_old, c_old = (a[sel] for a in (th, s_new, c_new, s_old, c_old))
    t = torch.from_numpy(th)
    s_mkl = torch.sin(t).numpy()
    c_mkl = torch.cos(t).numpy()
    x64 = th.astype(np.float64)
    s_cr = cr_from_f64(np.sin(x64))
    c_cr = cr_from_f64(np.cos(x64))
    # adjudicate the shipped value against long double where it differs from
    # the fp64-rounded reference (fp64 sin can sit within an ulp of a midpoint)
    non_cr = 0
    examples = []
    for got, ref, fn in ((s_new, s_cr, np.sin), (c_new, c_cr, np.cos)):
        d = np.nonzero(got != ref)[0]
        if d.size:
            ld = fn(th[d].astype(np.longdouble)).astype(np.float32)
            bad = got[d] != ld
            non_cr += int(bad.sum())
            examples += [float(v) for v in th[d][bad][:4]]
    eq = lambda a, b: (a.view(np.uint32) == b.view(np.uint32))  # noqa: E731
    return np.array([
        th.size,
        eq(s_new, s_mkl).sum(), eq(c_new, c_mkl).sum(), (eq(s_new, s_mkl) & eq(c_new, c_mkl)).sum(),
        eq(s_old, s_mkl).sum(), eq(c_old, c_mkl).sum(), (eq(s_old, s_mkl) & eq(c_old, c_mkl)).sum(),
        eq(s_cr, s_mkl).sum(), eq(c_cr, c_mkl).sum(),
        non_cr,
    ], np.int64), examples


def acos_chunk(first, n, step):
    a_glibc = orc.acosf_range(first, n)
    bits = (np.arange(n, dtype=np.uint64) + first).astype(np.uint32)
    x = bits.view(np.float32)
    if step > 1:
        x, a_glibc = x[::step], a_glibc[::step]
    a_mkl = torch.acos(torch.from_numpy(x)).numpy()
    a_cr = np.arccos(x.astype(np.float64)).astype(np.float32)
    eq = lambda a, b: (a.view(np.uint32) == b.view(np.uint32))  # noqa: E731
    return np.array([x.size, eq(a_glibc, a_mkl).sum(), eq(a_cr, a_mkl).sum(),
                     eq(a_glibc, a_cr).sum()], np.int64)


def uniform_sample():
    """The same comparisons over angles drawn uniformly in value (how headings
    and bearings are distributed), where the all-fp32 sweep is dominated by
    the tiny angles at which sin x = x and cos x = 1 are trivially exact."""
    g = np.random.default_rng(11)
    th = g.uniform(-np.pi, np.pi, 1 << 24).astype(np.float32)
    s_new, c_new = orc.sincos(th, 0)
    s_old, c_old = orc.sincos(th, 1)
    t = torch.from_numpy(th)
    s_mkl, c_mkl = torch.sin(t).numpy(), torch.cos(t).numpy()
    x = g.uniform(-1, 1, 1 << 24).astype(np.float32)
    a_mkl = torch.acos(torch.from_numpy(x)).numpy()
    a_glibc = orc.acosf(x)
    a_cr = np.arccos(x.astype(np.float64)).astype(np.float32)
    m = lambda a, b: float(np.mean(a.view(np.uint32) == b.view(np.uint32)))  # noqa: E731
    return {"samples": int(th.size),
            "shipped_fp64_sincos_vs_mkl": {"sin": m(s_new, s_mkl), "cos": m(c_new, c_mkl)},
            "round2_fp32_cephes_vs_mkl": {"sin": m(s_old, s_mkl), "cos": m(c_old, c_mkl)},
            "acos_uniform[-1,1]": {"glibc_acosf_vs_mkl": m(a_glibc, a_mkl),
                                   "correctly_rounded_vs_mkl": m(a_cr, a_mkl)}}


def ranges(hi_bits):
    """[+0 .. hi] and [-0 .. -hi] as (first, n) chunks of consecutive bit patterns."""
    out = []
    for base in (0, 0x80000000):
        first, last = base, base + hi_bits
        while first <= last:
            n = min(CHUNK, last - first + 1)
            out.append((first, n))
            first += n
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    step = 64 if a.quick else 1
    torch.set_num_threads(1)   # parallel over chunks instead
    t0 = time.time()
    fns, mode, path = vml()
    ident = identity_check(fns)
    print("identity torch == MKL VML:", json.dumps(ident))

    tot = np.zeros(10, np.int64)
    ex = []
    with ThreadPoolExecutor(8) as pool:
        for cnt, e in pool.map(lambda fr: sweep_chunk(fr[0], fr[1], step), ranges(PI_BITS)):
            tot += cnt
            ex += e
    n = int(tot[0])
    sweep = {
        "inputs": n,
        "range": "every fp32 in [-pi, pi] incl. +-0 (pi rounded up, the clamp bound)",
        "shipped_fp64_sincos_vs_mkl": {"sin": tot[1] / n, "cos": tot[2] / n, "both": tot[3] / n},
        "round2_fp32_cephes_vs_mkl": {"sin": tot[4] / n, "cos": tot[5] / n, "both": tot[6] / n},
        "correctly_rounded_vs_mkl": {"sin": tot[7] / n, "cos": tot[8] / n},
        "shipped_not_correctly_rounded": int(tot[9]),
        "shipped_not_correctly_rounded_examples": ex[:8],
    }
    sweep = json.loads(json.dumps(sweep, default=float))
    print("sin/cos sweep:", json.dumps(sweep, indent=1))

    tot = np.zeros(4, np.int64)
    with ThreadPoolExecutor(8) as pool:
        for cnt in pool.map(lambda fr: acos_chunk(fr[0], fr[1], step), ranges(ONE_BITS)):
            tot += cnt
    n = int(tot[0])
    acos = {"inputs": n, "range": "every fp32 in [-1, 1] (the clamped dot product, :280-281)",
            "glibc_acosf_vs_mkl": tot[1] / n, "correctly_rounded_vs_mkl": tot[2] / n,
            "glibc_acosf_vs_correctly_rounded": tot[3] / n}
    acos = json.loads(json.dumps(acos, default=float))
    print("acos sweep:", json.dumps(acos, indent=1))
    uni = uniform_sample()
    print("uniform sample:", json.dumps(uni, indent=1))
    print(f"{time.time() - t0:.0f} s")
    if a.quick:
        return
    mpath = os.path.join(HERE, "MANIFEST.json")
    with open(mpath) as fh:
        man = json.load(fh)
    man["libm"] = {
        "what": "the reference's CPU torch.sin/cos/acos (environment.py:131-137, 286) are "
                "MKL VML vsSin/vsCos/vsAcos in this torch build; generated by "
                "tests/golden/libm_check.py",
        "torch": torch.__version__,
        "mkl": torch.backends.mkl.is_available() and torch.__config__.show().split(
            "Math Kernel Library Version ")[1].split(" ")[0],
        "cpu_capability": torch.backends.cpu.get_cpu_capability(),
        "vml_mode": mode,
        "vml_library": os.path.relpath(path, os.path.dirname(torch.__file__)),
        "torch_equals_vml": ident,
        "sincos_sweep": sweep,
        "acos_sweep": acos,
        "uniform_sample": uni,
    }
    with open(mpath, "w") as fh:
        json.dump(man, fh, indent=1, sort_keys=True)
        fh.write("\n")
    print("wrote", mpath)


if __name__ == "__main__":
    main()
