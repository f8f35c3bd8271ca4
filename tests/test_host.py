"""Host-side logic of the drop-in Env that needs no GPU: the step-output
recycling rule (marl-nav_amd/environment.py _OutputSet)."""
import importlib

import numpy as np

import torch

envmod = importlib.import_module("marl-nav_amd.environment")


class _Stub:
    """The attributes _OutputSet reads from an Env."""
    _obs_shape = (10, 3, 12)
    device = torch.device("cpu")
    _obs_norm_buffers = None
    _split = [1, 1, 3, 3, 2, 2]
    _normalizer = None
    _wrap_obs = envmod.Env._wrap_obs


def test_output_set_layout():
    s = envmod._OutputSet(_Stub())
    assert s.packed.shape == (10, 3, 12) and s.packed.dtype == torch.float32
    assert s.reward.shape == (10,) and s.terminated.dtype == torch.bool
    assert [tuple(f.shape) for f in s.obs] == [(10, 3, 1), (10, 3, 1), (10, 3, 3), (10, 3, 3),
                                               (10, 3, 2), (10, 3, 2)]
    # one allocation, disjoint regions
    regions = sorted((t.data_ptr(), t.data_ptr() + t.numel() * t.element_size())
                     for t in (s.packed, s.reward, s.terminated, s.truncated))
    assert all(a[1] <= b[0] for a, b in zip(regions, regions[1:]))
    assert s.obs._packed is s.packed


def test_output_set_is_free_only_when_unreferenced():
    s = envmod._OutputSet(_Stub())
    s.arm()
    assert s.free()
    held = [lambda: s.reward, lambda: s.obs, lambda: s.obs[3], lambda: s.obs.target_angle[2:4],
            lambda: s.packed.view(-1), lambda: s.truncated[1:], lambda: (s.obs, s.reward)]
    for make in held:
        x = make()
        assert not s.free()
        del x
        assert s.free()


def test_cli_mirrors_reference_arguments():
    """python -m marlnav_amd takes the reference's arguments with its
    defaults (marlnav/__main__.py:49-132; utils.default_args restates them)."""
    cli = importlib.import_module("marl-nav_amd.cli")
    utils = importlib.import_module("marl-nav_amd.utils")
    ns = vars(cli.build_parser().parse_args([]))
    ref = vars(utils.default_args())
    for k, v in ref.items():
        assert ns[k] == v, k
    assert cli.main([]) == 2          # training stays in the reference
    assert cli.main(["-re"]) == 2     # and so does rendering


def test_comparators_see_non_finite_values():
    """The parity comparators must not accept NaN against a number (or the
    other way round), nor an infinity of the other sign; NaN facing NaN and
    equal infinities pass."""
    import pytest as _pt
    from conftest import OBS_FIELDS, assert_obs_close, assert_states_close, assert_vec_close
    nan, inf = float("nan"), float("inf")
    assert_vec_close([1.0, nan, inf, -inf], [1.0, nan, inf, -inf])
    for got, want in (([nan], [1.0]), ([1.0], [nan]), ([inf], [-inf]), ([inf], [1e38]),
                      ([1.0], [inf])):
        with _pt.raises(AssertionError):
            assert_vec_close(got, want)
    base = {f: np.ones((2, 3, 1)) for f in OBS_FIELDS}
    for f in OBS_FIELDS:
        bad = [base[g].copy() for g in OBS_FIELDS]
        bad[OBS_FIELDS.index(f)][1, 2, 0] = nan
        with _pt.raises(AssertionError):
            assert_obs_close(bad, base, prefix="")
        with _pt.raises(AssertionError):
            assert_obs_close(bad, base, prefix="", exact_distances=True)
    st = np.ones((2, 3, 5))
    st2 = st.copy()
    st2[0, 1, 3] = nan
    with _pt.raises(AssertionError):
        assert_states_close(st2, st)
    st3 = st.copy()
    st3[1, 0, 2] = inf
    with _pt.raises(AssertionError):
        assert_states_close(st3, st)
    assert_states_close(st3, st3.copy())
