"""Shared test plumbing: the `gpu` marker, golden-fixture loading, and the
mapping from fixture metadata to the kernel's parameter struct."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
OBS_FIELDS = ("target_angle", "target_distance", "obstacles_angles",
              "obstacles_distances", "others_angles", "others_distances")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")


def manifest():
    with open(os.path.join(GOLDEN, "MANIFEST.json")) as fh:
        return json.load(fh)


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def meta(name):
    return manifest()["files"][name + ".npz"]


def env_values(m):
    """Fixture metadata -> Env-attribute-named values for make_cparams."""
    return {"min_speed": m["min_speed"], "max_speed": m["max_speed"],
            "min_accel": m["min_accel"], "max_accel": m["max_accel"],
            "_risk_factor": m["risk_factor"], "_distance_factor": m["distance_factor"],
            "_heading_factor": m["heading_factor"], "_target_factor": m["target_factor"],
            "_soft_factor": m["soft_factor"], "_bond_factor": m["bond_factor"],
            "episode_len": m["episode_len"]}


def cli_args(**over):
    """The reference CLI defaults (marlnav/__main__.py:49-132)."""
    import marlnav_amd
    return marlnav_amd.default_args(**over)


ANGLE_FIELDS = ("target_angle", "obstacles_angles", "others_angles")
DIST_FIELDS = ("target_distance", "obstacles_distances", "others_distances")

# Tolerances (north_star: obs and rewards within 1e-5 relative). Angles have
# no absolute floor: the heading's sin/cos is correctly rounded on both the
# kernel and the oracle side (the reference's MKL VML sin/cos agrees with the
# correctly rounded value on 95% of headings; tests/golden/libm_check.py), and
# every golden angle entry is within RTOL of the reference's.
RTOL = 1e-5


def _close_mask(a, e, rtol, atol):
    """Elementwise 'outside tolerance' for float arrays that may hold
    non-finite values: NaN must face NaN, +-inf must equal exactly, finite
    values are compared with |a - e| <= atol + rtol*|e| (never silently true
    for NaN, unlike the bare comparison)."""
    a = np.asarray(a, np.float64)
    e = np.asarray(e, np.float64)
    an, en = np.isnan(a), np.isnan(e)
    ai, ei = np.isinf(a), np.isinf(e)
    fin = ~(an | en | ai | ei)
    bad = (an != en) | ((ai | ei) & ~(an | en) & (a != e))
    with np.errstate(invalid="ignore"):
        bad |= fin & (np.abs(a - e) > atol + rtol * np.abs(e))
    return a, e, bad


def _report(what, a, e, bad):
    i = np.argwhere(bad)[0].tolist()
    return (f"{what}: {int(bad.sum())} of {bad.size} outside tol; first at {i}: "
            f"got {a[tuple(i)]!r} want {e[tuple(i)]!r}")


def assert_bits_equal(a, e, what=""):
    """Float arrays equal bit for bit (+0 and -0 differ), except that a NaN
    must face a NaN of any payload."""
    a = np.ascontiguousarray(a, np.float32)
    e = np.ascontiguousarray(e, np.float32)
    assert a.shape == e.shape, f"{what}: shape {a.shape} vs {e.shape}"
    an, en = np.isnan(a), np.isnan(e)
    bad = (an != en) | (~an & (a.view(np.uint32) != e.view(np.uint32)))
    assert not bad.any(), _report(what + " (bit-exact)", a, e, bad)


def assert_obs_close(actual_fields, expected, prefix="obs_", rtol=RTOL, where="",
                     exact_distances=False, angle_atol=0.0, exact=False):
    """The six Observations fields against expected ones: every field within
    rtol (angles with an absolute ``angle_atol`` only where a caller passes
    one), distances bit-exact with ``exact_distances`` (the oracle
    comparisons: both sides compute sqrtf(fmaf(dy,dy,dx*dx)),
    environment.py:271-274); NaN/inf positions must match in every field.
    ``exact``: every field bit for bit (the kernel against the oracle, whose
    bearings use the kernel's own acos, oracle/marlnav_oracle.c acos_device)."""
    for f, a in zip(OBS_FIELDS, actual_fields):
        e = expected[prefix + f] if isinstance(expected, dict) or hasattr(expected, "files") \
            else expected[f]
        if exact:
            assert_bits_equal(a, e, f"{where} {f}")
            continue
        if exact_distances and f in DIST_FIELDS:
            np.testing.assert_array_equal(np.asarray(a), np.asarray(e), f"{where} {f}")
            continue
        atol = angle_atol if f in ANGLE_FIELDS else 0.0
        a, e, bad = _close_mask(a, e, rtol, atol)
        assert not bad.any(), _report(f"{where} {f}", a, e, bad)


def assert_vec_close(a, e, rtol=RTOL, atol=0.0, what=""):
    a, e, bad = _close_mask(a, e, rtol, atol)
    assert not bad.any(), _report(what, a, e, bad)


# (test, compared against, angle entries, entries not bit-equal, entries
# beyond RTOL, worst relative error), filled by record_angle_stats and printed
# in the session summary
ANGLE_STATS = []


def record_angle_stats(test, against, actual_fields, expected_fields):
    n_ne, n_beyond, worst = angle_error_stats(actual_fields, expected_fields)
    n = sum(int(np.asarray(a).size) for f, a in zip(OBS_FIELDS, actual_fields)
            if f in ANGLE_FIELDS)
    ANGLE_STATS.append((test, against, n, n_ne, n_beyond, worst))
    return n_beyond, worst


# Threshold proximity: the reward and terminal logic
# compares fp32 values with fixed thresholds (environment.py:172-177 the angle
# cap, :184-257 risk / collision / band / target / heading), so an output that
# is 1 ulp away from the reference's can flip a flag only when it sits within
# a few ulp of a threshold. Per comparison, how many entries do. Geometry:
# environment.py:56-68 (marlnav_amd.environment.GEOMETRY).
THRESH_STATS = {}
THRESH_ULPS = 4


def _near(x, t, ulps=THRESH_ULPS):
    """entries of x within `ulps` fp32 ulps of the threshold t (either sign of
    t for |x| comparisons is the caller's choice)"""
    x = np.asarray(x, np.float32).ravel()
    x = x[np.isfinite(x)]
    xi = x.view(np.int32).astype(np.int64)
    ti = np.float32(t).view(np.int32).astype(np.int64)
    return int(np.count_nonzero((np.sign(x) == np.sign(np.float32(t))) & (np.abs(xi - ti) <= ulps)))


def record_threshold_stats(test, fields, geometry=None):
    """fields: the six Observations arrays in OBS_FIELDS order. Counts target
    bearings within THRESH_ULPS of +-max_angle_diff (the heading term,
    environment.py:253-257) and distances within THRESH_ULPS of each distance
    threshold that reads them, and of the angle cap."""
    import math
    g = {'_ob_risk_dist': 60., '_ag_risk_dist': 15., '_ob_coll_dist': 50., '_ag_coll_dist': 5.,
         '_agents_min_d': 30., '_agents_max_d': 50., '_max_angle_diff': math.pi / 8,
         '_target_radius': 30., '_cap_distance': 0.1}
    g.update(geometry or {})
    f = dict(zip(OBS_FIELDS, fields))
    ta, td = f["target_angle"], f["target_distance"]
    od, gd = f["obstacles_distances"], f["others_distances"]
    mad = float(np.float32(g['_max_angle_diff']))
    c = THRESH_STATS.setdefault(test, {})
    add = lambda k, v: c.__setitem__(k, c.get(k, 0) + v)
    add("n_rows", int(np.asarray(ta).size))
    add("heading |ta|~max_angle_diff", _near(ta, mad) + _near(ta, -mad))
    add("target_dist~target_radius", _near(td, g['_target_radius']))
    add("obst_dist~ob_risk", _near(od, g['_ob_risk_dist']))
    add("obst_dist~ob_coll", _near(od, g['_ob_coll_dist']))
    add("other_dist~ag_risk", _near(gd, g['_ag_risk_dist']))
    add("other_dist~ag_coll", _near(gd, g['_ag_coll_dist']))
    add("other_dist~band_min", _near(gd, g['_agents_min_d']))
    add("other_dist~band_max", _near(gd, g['_agents_max_d']))
    add("any_dist~cap", sum(_near(x, g['_cap_distance']) for x in (td, od, gd)))


def pytest_terminal_summary(terminalreporter):
    if THRESH_STATS:
        terminalreporter.write_sep(
            "-", f"threshold proximity: entries within {THRESH_ULPS} ulp of a reward/terminal threshold")
        for test, c in sorted(THRESH_STATS.items()):
            near = {k: v for k, v in c.items() if k != "n_rows"}
            terminalreporter.write_line(
                f"{test}: {c['n_rows']} rows; " + ", ".join(f"{k} {v}" for k, v in near.items()))
    if TRAJ_STATS:
        terminalreporter.write_sep("-", "trajectory angles away from 0 and pi: largest deviation (rad)")
        for k, v in sorted(TRAJ_STATS.items()):
            terminalreporter.write_line(f"{k}: {v:.3g}")
    if not ANGLE_STATS:
        return
    agg = {}
    for test, against, n, n_ne, n_beyond, worst in ANGLE_STATS:
        a = agg.setdefault((test, against), [0, 0, 0, 0.0])
        a[0] += n
        a[1] += n_ne
        a[2] += n_beyond
        a[3] = max(a[3], worst)
    tr = terminalreporter
    tr.write_sep("-", "angle fields: entries not bit-equal, beyond RTOL, worst relative error")
    for (test, against), (n, n_ne, n_beyond, worst) in sorted(agg.items()):
        tr.write_line(f"{test} vs {against}: {n} angles, {n_ne} not bit-equal, {n_beyond} "
                      f"beyond rtol {RTOL:g} (no absolute floor), worst rel err {worst:.3g}")


def angle_error_stats(actual_fields, expected_fields):
    """(entries not bit-equal, entries beyond RTOL, worst relative error over
    every finite entry with a nonzero expected value; an expected 0 with a
    nonzero actual counts as beyond)."""
    n_ne, n_beyond, worst = 0, 0, 0.0
    for f, a, e in zip(OBS_FIELDS, actual_fields, expected_fields):
        if f not in ANGLE_FIELDS:
            continue
        a = np.asarray(a, np.float64)
        e = np.asarray(e, np.float64)
        fin = np.isfinite(a) & np.isfinite(e)
        d = np.abs(a - e)[fin]
        ea = np.abs(e[fin])
        n_ne += int((d > 0).sum())
        n_beyond += int((d > RTOL * ea).sum())
        nz = ea > 0
        if nz.any():
            worst = max(worst, float((d[nz] / ea[nz]).max()))
    return n_ne, n_beyond, worst


def assert_states_close(a, e, what="states"):
    """Agent states (..., 5): positions and speed within rtol; the heading
    vector within 1e-6 of its own magnitude (a 1-ulp sin/cos difference on a
    component that cancels to ~0 is not a relative error of that component)."""
    a = np.asarray(a, np.float64)
    e = np.asarray(e, np.float64)
    assert np.array_equal(np.isnan(a), np.isnan(e)), f"{what}: NaN pattern differs"
    assert_vec_close(a[..., [0, 1, 4]], e[..., [0, 1, 4]], what=what + "[pos,speed]")
    mag = np.linalg.norm(e[..., 2:4], axis=-1, keepdims=True)
    with np.errstate(invalid="ignore"):
        bad = np.abs(a[..., 2:4] - e[..., 2:4]) > 1e-6 * np.maximum(mag, 1e-30)
    bad &= np.isfinite(e[..., 2:4]) & np.isfinite(mag)
    bad |= np.isfinite(a[..., 2:4]) != np.isfinite(e[..., 2:4])
    bad |= np.isinf(e[..., 2:4]) & (a[..., 2:4] != e[..., 2:4])
    assert not bad.any(), f"{what}[dir]: {bad.sum()} outside 1e-6*|dir|"


@pytest.fixture(scope="session")
def pkg():
    import marlnav_amd
    return marlnav_amd


def angle_columns(A, O):
    """Indices of the angle features in a packed (.., D) observation row."""
    return [0] + [2 + j for j in range(O)] + [2 + 2 * O + k for k in range(A - 1)]


TRAJ_STATS = {}


def assert_traj_obs_close(got, want, A, O, angle_scale=1.0, what="", angle_tol=1e-4):
    """Packed observations of a multi-step trajectory against the
    reference's. A heading carries the sin/cos differences of every step (the
    reference's MKL sin/cos vs the correctly rounded one, 5% of the values
    1 ulp apart), and acos is ill-conditioned next to 0 and pi (acos(1 - k
    ulp) moves by ~3e-4 rad per ulp of the dot product there), so angles
    (packed value * angle_scale, in rad) are compared twice: through their
    cosine, i.e. the clamped dot product the angle is acos of (within 1e-5
    absolute), and - where the reference bearing is clearly away from 0 and pi
    (|sin| > 1e-2, so its sign is observable) - by sign and value (within
    ``angle_tol`` rad). Every other feature within rtol 1e-5 (+ 2e-5 absolute
    for normalised values near 0). NaN must face NaN."""
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    ang = np.zeros(got.shape[-1], bool)
    ang[angle_columns(A, O)] = True
    assert_vec_close(got[..., ~ang], want[..., ~ang], rtol=RTOL, atol=2e-5, what=what + " non-angles")
    ga, wa = got[..., ang] * angle_scale, want[..., ang] * angle_scale
    assert_vec_close(np.cos(ga), np.cos(wa), rtol=0.0, atol=1e-5, what=what + " cos(angle)")
    with np.errstate(invalid="ignore"):
        away = np.isfinite(wa) & (np.abs(np.sin(wa)) > 1e-2)
    assert np.array_equal(np.sign(ga[away]), np.sign(wa[away])), what + " angle sign"
    dev = np.abs(ga[away] - wa[away])
    if dev.size:
        TRAJ_STATS[what.split()[0]] = max(TRAJ_STATS.get(what.split()[0], 0.0), float(dev.max()))
    assert not (dev > angle_tol).any(), f"{what} angle: {int((dev > angle_tol).sum())} beyond {angle_tol}"
