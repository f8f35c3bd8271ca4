"""Distribution checks of the native re-init draws (the Philox stream of
``rng='native'``) against the law of the reference's sampler,
TriangleIntitializer (marlnav/utils.py:381-398):

* obstacles: x = range_x * (u - 0.5) + mean_x, y likewise, u = torch.rand,
  i.e. u uniform on the 24-bit grid {k * 2^-24 : 0 <= k < 2^24}, every
  operation rounded to fp32 (the defaults: x in [500, 1000], y in [250, 500]);
* noisy agents (utils.py:381-388): position noise ags_dist * N(0, ags_std I)
  (MultivariateNormal with covariance diag(ags_std)), heading angle
  angle_range * (u - 0.5).

The native stream cannot reproduce torch's Mersenne-Twister draws, so its
parity with the reference is distributional:
every value must lie on the exact image of the 24-bit grid under the
reference's fp32 map, and the draws must pass moment, chi-square and KS
tests against the uniform law and a two-sample KS test against draws of the
reference's own sampler (the host reference-RNG mode, pinned draw for draw to
the reference by fixture F4, tests/golden/triangle_rng.npz).

The draws are deterministic functions of (seed, step, env), so these tests
are deterministic: a p-value threshold is a fixed pass/fail, not a flake rate.
"""
import numpy as np
from scipy import stats

P_MIN = 1e-6          # smallest acceptable p-value of each test
GRID = 1 << 24        # torch.rand's fp32 grid


def grid_image(rng, mean):
    """fl(fl(rng * fl(u - 0.5)) + mean) for every u = k * 2^-24 in [0, 1):
    the values the reference's obstacle sampler can produce (monotone)."""
    u = np.arange(GRID, dtype=np.float32) * np.float32(2.0 ** -24)  # exact
    x = np.float32(rng) * (u - np.float32(0.5)) + np.float32(mean)
    assert x.dtype == np.float32 and np.all(np.diff(x) >= 0)
    return x


def grid_u(vals, image):
    """Check every value lies on `image` and return its grid coordinate
    u = k * 2^-24 (the first k that maps to it)."""
    vals = np.ascontiguousarray(vals, np.float32).ravel()
    k = np.searchsorted(image, vals)
    on = (k < GRID) & (image[np.minimum(k, GRID - 1)] == vals)
    assert on.all(), f"{(~on).sum()} of {vals.size} draws off the 24-bit grid image, e.g. {vals[~on][:5]}"
    return k.astype(np.float64) / GRID


def check_uniform(u, what, n_bins=1024):
    """u (float64 in [0, 1)): mean, variance, chi-square on n_bins, KS."""
    n = u.size
    se_mean = np.sqrt(1.0 / 12.0 / n)
    assert abs(u.mean() - 0.5) < 6 * se_mean, (what, u.mean())
    se_var = np.sqrt((1.0 / 80.0 - 1.0 / 144.0) / n)
    assert abs(u.var() - 1.0 / 12.0) < 6 * se_var, (what, u.var())
    counts = np.bincount(np.minimum((u * n_bins).astype(np.int64), n_bins - 1), minlength=n_bins)
    chi = stats.chisquare(counts)
    ks = stats.kstest(u, "uniform")
    assert chi.pvalue > P_MIN, (what, "chi2", chi)
    assert ks.pvalue > P_MIN, (what, "ks", ks)
    return {"n": n, "mean": float(u.mean()), "var": float(u.var()),
            "chi2_p": float(chi.pvalue), "ks_p": float(ks.pvalue)}


def check_same_law(a, b, what):
    """Two-sample KS of the native draws `a` against reference draws `b`."""
    r = stats.ks_2samp(np.ravel(a), np.ravel(b))
    assert r.pvalue > P_MIN, (what, r)
    return float(r.pvalue)


def check_uncorrelated(x, y, what):
    """Pearson correlation of paired samples within 6 standard errors of 0."""
    x = np.ravel(x).astype(np.float64)
    y = np.ravel(y).astype(np.float64)
    r = np.corrcoef(x, y)[0, 1]
    assert abs(r) < 6.0 / np.sqrt(x.size), (what, r)
    return float(r)


def check_obstacles(ob, rx, mx, ry, my, ref=None, what="obstacles"):
    """ob (P, O, 2) native draws; ref (Q, O, 2) reference draws or None.
    Returns a dict of the statistics (printed by the tests)."""
    ob = np.asarray(ob, np.float32)
    out = {}
    ux = grid_u(ob[..., 0], grid_image(rx, mx)).reshape(ob.shape[:2])
    uy = grid_u(ob[..., 1], grid_image(ry, my)).reshape(ob.shape[:2])
    out["x"] = check_uniform(ux.ravel(), what + " x")
    out["y"] = check_uniform(uy.ravel(), what + " y")
    out["r_xy"] = check_uncorrelated(ux, uy, what + " x-y")
    if ob.shape[1] > 1:  # consecutive obstacles of one env
        out["r_obst"] = check_uncorrelated(ux[:, :-1], ux[:, 1:], what + " obstacle j, j+1")
        out["r_obst_y"] = check_uncorrelated(uy[:, :-1], uy[:, 1:], what + " obstacle j, j+1 (y)")
    out["r_env"] = check_uncorrelated(ux[:-1], ux[1:], what + " env e, e+1")
    if ref is not None:
        ref = np.asarray(ref, np.float32)
        out["ks2_x"] = check_same_law(ob[..., 0], ref[..., 0], what + " x vs reference")
        out["ks2_y"] = check_same_law(ob[..., 1], ref[..., 1], what + " y vs reference")
    return out


def check_noisy_agents(states, formation, ags_dist, ags_std, angle_range, ref=None,
                       what="noisy agents"):
    """states (P, A, 5) of fresh noisy envs; formation (A, 5). Position noise
    / (ags_dist * sqrt(ags_std)) ~ N(0, 1) per coordinate; heading angle
    (from the rotated formation direction (1, 0)) / angle_range + 0.5 ~ U(0, 1)."""
    st = np.asarray(states, np.float64)
    fm = np.asarray(formation, np.float64)
    z = (st[..., :2] - fm[None, :, :2]) / (ags_dist * np.sqrt(ags_std))
    out = {}
    for c in range(2):
        zc = z[..., c].ravel()
        n = zc.size
        assert abs(zc.mean()) < 6 / np.sqrt(n), (what, c, zc.mean())
        assert abs(zc.var() - 1.0) < 6 * np.sqrt(2.0 / n), (what, c, zc.var())
        ks = stats.kstest(zc, "norm")
        assert ks.pvalue > P_MIN, (what, c, ks)
        out[f"ks_norm_{c}"] = float(ks.pvalue)
    out["r_xy"] = check_uncorrelated(z[..., 0], z[..., 1], what + " noise x-y")
    ang = np.arctan2(st[..., 3], st[..., 2])
    ua = ang / angle_range + 0.5
    # sin/cos of an fp32 angle and the atan2 back: the angle is recovered to
    # ~1e-7 rad, far inside any bin; KS on the continuous law
    ks = stats.kstest(ua.ravel(), "uniform")
    assert ks.pvalue > P_MIN, (what, "angle", ks)
    out["ks_angle"] = float(ks.pvalue)
    out["r_pos_angle"] = check_uncorrelated(z[..., 0], ua, what + " noise-angle")
    if ref is not None:
        zr = (np.asarray(ref, np.float64)[..., :2] - fm[None, :, :2]) / (ags_dist * np.sqrt(ags_std))
        out["ks2_pos"] = check_same_law(z[..., 0], zr[..., 0], what + " noise vs reference")
    return out
