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

# Tolerances (north_star: obs and rewards within 1e-5 relative). Angles get an
# absolute floor of 2e-6 rad: acos is ill-conditioned near 0 and pi, where a
# 1-ulp difference of the heading (torch's SLEEF sin/cos vs a correctly
# rounded one) is amplified; away from there the relative bound binds.
RTOL = 1e-5
ANGLE_ATOL = 2e-6


def assert_obs_close(actual_fields, expected, prefix="obs_", rtol=RTOL, where=""):
    for f, a in zip(OBS_FIELDS, actual_fields):
        e = expected[prefix + f] if isinstance(expected, dict) or hasattr(expected, "files") \
            else expected[f]
        a = np.asarray(a, np.float64)
        e = np.asarray(e, np.float64)
        atol = ANGLE_ATOL if f in ANGLE_FIELDS else 0.0
        bad = np.abs(a - e) > atol + rtol * np.abs(e)
        assert not bad.any(), (
            f"{where} {f}: {bad.sum()} of {bad.size} outside tol; first at "
            f"{np.argwhere(bad)[0].tolist()}: got {a[bad][0]!r} want {e[bad][0]!r}")


def assert_vec_close(a, e, rtol=RTOL, atol=0.0, what=""):
    a = np.asarray(a, np.float64)
    e = np.asarray(e, np.float64)
    bad = np.abs(a - e) > atol + rtol * np.abs(e)
    assert not bad.any(), (f"{what}: {bad.sum()} of {bad.size} outside tol; first at "
                           f"{np.argwhere(bad)[0].tolist()}: got {a[bad][0]!r} want {e[bad][0]!r}")


def assert_states_close(a, e, what="states"):
    """Agent states (..., 5): positions and speed within rtol; the heading
    vector within 1e-6 of its own magnitude (a 1-ulp sin/cos difference on a
    component that cancels to ~0 is not a relative error of that component)."""
    a = np.asarray(a, np.float64)
    e = np.asarray(e, np.float64)
    assert_vec_close(a[..., [0, 1, 4]], e[..., [0, 1, 4]], what=what + "[pos,speed]")
    mag = np.linalg.norm(e[..., 2:4], axis=-1, keepdims=True)
    bad = np.abs(a[..., 2:4] - e[..., 2:4]) > 1e-6 * np.maximum(mag, 1e-30)
    assert not bad.any(), f"{what}[dir]: {bad.sum()} outside 1e-6*|dir|"


@pytest.fixture(scope="session")
def pkg():
    import marlnav_amd
    return marlnav_amd
