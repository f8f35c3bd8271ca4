"""Host-side logic of the drop-in Env that needs no GPU: the step-output
recycling rule (marl-nav_amd/environment.py _OutputSet)."""
import importlib

import numpy as np

import torch

envmod = importlib.import_module("marl-nav_amd.environment")


class _Stub:
    """The attributes _new_output_set reads from an Env."""
    _obs_shape = (10, 3, 12)
    device = torch.device("cpu")
    _obs_norm_buffers = None
    _split = [1, 1, 3, 3, 2, 2]
    _normalizer = None
    _wrap_obs = envmod.Env._wrap_obs


def test_output_set_layout():
    obs, reward, term, trunc, packed, norm = envmod._new_output_set(_Stub())
    assert norm is None
    assert packed.shape == (10, 3, 12) and packed.dtype == torch.float32
    assert reward.shape == (10,) and term.dtype == torch.bool
    assert [tuple(f.shape) for f in obs] == [(10, 3, 1), (10, 3, 1), (10, 3, 3), (10, 3, 3),
                                             (10, 3, 2), (10, 3, 2)]
    # one allocation, disjoint regions
    regions = sorted((t.data_ptr(), t.data_ptr() + t.numel() * t.element_size())
                     for t in (packed, reward, term, trunc))
    assert all(a[1] <= b[0] for a, b in zip(regions, regions[1:]))
    assert obs._packed is packed


def _cpu_engine(calls):
    """The native host engine with a stand-in step function (records the
    output pointers it is given, returns 0) and CPU tensors: exercises the
    output-set pool without a GPU."""
    import ctypes
    abi = importlib.import_module("marl-nav_amd.abi")
    host = abi.load_host()
    proto = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.POINTER(abi.MarlnavStepBuffers), ctypes.c_uint64,
                             ctypes.c_void_p)

    def fake_step(d, p, b, idx, stream):
        calls.append((b.contents.obs, idx))
        return 0
    cb = proto(fake_step)
    stub = _Stub()
    eng = host.Engine(abi.fn_addr(cb), 0, lambda i: 0, -1,
                      lambda: envmod._new_output_set(stub), lambda a: None)
    dims = abi.MarlnavDims(num_parallel=10, num_agents=3, num_obstacles=3, obstacle_stride=3)
    eng.configure(bytes(dims), bytes(abi.MarlnavParams()), bytes(abi.MarlnavStepBuffers()), True)
    return eng, cb


def test_engine_recycles_an_output_set_only_when_unreferenced():
    calls = []
    eng, cb = _cpu_engine(calls)
    first = eng.launch(0, None, 0)
    obs, rew, term, trunc = first
    ptr0 = calls[-1][0]
    del first, obs, rew, term, trunc
    # nothing held: after another step the first set is reused (never the
    # set of the previous step)
    eng.launch(0, None, 0)
    eng.launch(0, None, 0)
    assert calls[-1][0] == ptr0
    assert [c[1] for c in calls] == [1, 2, 3]      # step index advances per launch
    # any kept object or view keeps its set out of the pool's reuse
    for k in range(8):
        out = eng.launch(0, None, 0)
        keep = [lambda o: o[1], lambda o: o[0], lambda o: o[0][3], lambda o: o[0].target_angle[2:4],
                lambda o: o[0]._packed.view(-1), lambda o: o[3][1:], lambda o: o[2],
                lambda o: o[0]._packed][k](out)
        kept_ptr = calls[-1][0]
        del out
        for _ in range(6):
            eng.launch(0, None, 0)
            assert calls[-1][0] != kept_ptr, k
        del keep
    assert len(eng.pool_info()) <= 4


def test_engine_fast_path_falls_back_for_other_actions():
    calls = []
    _, cb = _cpu_engine(calls)
    seen = []
    abi = importlib.import_module("marl-nav_amd.abi")
    host = abi.load_host()
    stub = _Stub()
    eng = host.Engine(abi.fn_addr(cb), 0, lambda i: 0, 0,
                      lambda: envmod._new_output_set(stub), lambda a: seen.append(a) or "slow")
    dims = abi.MarlnavDims(num_parallel=10, num_agents=3, num_obstacles=3, obstacle_stride=3)
    eng.configure(bytes(dims), bytes(abi.MarlnavParams()), bytes(abi.MarlnavStepBuffers()), True)
    # CPU tensors are never taken by the fast path (it wants the env's HIP device)
    assert eng(torch.zeros(10, 3, 2)) == "slow" and len(seen) == 1
    assert eng([1, 2]) == "slow"
    eng.fast_ok = 0
    assert eng(torch.zeros(10, 3, 2)) == "slow"
    assert calls == []


def test_engine_reports_held_state_tensors():
    """Copy-on-write rule for the tensors a step writes (environment.py:79-83
    and :219 rebind them): obstacles / target / step_num /
    terminates count as held once anything beyond their owner's attribute and
    the engine refers to them, the two state buffers (which only the engine
    holds: Env.states asks it) once anything at all does; a view sharing the
    storage counts too; a held tensor keeps steps off the fast path."""
    calls = []
    eng, cb = _cpu_engine(calls)

    class Owner:
        pass
    o = Owner()
    o.ob, o.tg = torch.zeros(10, 3, 2), torch.zeros(10, 1, 2)
    o.sn, o.tm = torch.zeros(10), torch.zeros(10, dtype=torch.bool)
    track = lambda s, alt: eng.track_state(s, o.ob, o.tg, o.sn, o.tm, alt)  # noqa: E731
    none = (False,) * 6
    track(torch.zeros(10, 3, 5), torch.zeros(10, 3, 5))
    assert eng.shared_state() == none
    s = eng.states()
    assert eng.shared_state() == (True, False, False, False, False, False)
    del s
    a = eng.states_alt()[2:]
    assert eng.shared_state() == (False, False, False, False, False, True)
    del a
    v = o.tg[:, 0]
    assert eng.shared_state() == (False, False, True, False, False, False)
    del v
    lst = [o.ob]
    assert eng.shared_state() == (False, True, False, False, False, False)
    del lst
    sn = o.sn
    assert eng.shared_state() == (False, False, False, True, False, False)
    del sn
    tm = o.tm[3:]
    assert eng.shared_state() == (False, False, False, False, True, False)
    del tm
    assert eng.shared_state() == none
    # a launch swaps the state buffers: the one written becomes current
    cur, alt = eng.states().data_ptr(), eng.states_alt().data_ptr()
    eng.launch(0, None, 0)
    assert (eng.states().data_ptr(), eng.states_alt().data_ptr()) == (alt, cur)
    # re-tracking releases the old tensors; no second buffer: in place
    track(torch.zeros(10, 3, 5), None)
    assert eng.shared_state() == none and eng.states_alt() is None
    p0 = eng.states().data_ptr()
    eng.launch(0, None, 0)
    assert eng.states().data_ptr() == p0


def test_dlpack_export_counts_as_a_holder():
    """INTEGRATION.md's holder contract: a raw-pointer consumer must hold a
    tensor reference. A DLPack export (torch.utils.dlpack.to_dlpack) does -
    its capsule keeps the storage - so an exported output set is not
    recycled and an exported state tensor is not written in place, until the
    capsule is gone."""
    from torch.utils.dlpack import to_dlpack
    calls = []
    eng, cb = _cpu_engine(calls)
    out = eng.launch(0, None, 0)
    cap = to_dlpack(out[0]._packed)
    ptr = calls[-1][0]
    del out
    for _ in range(6):
        eng.launch(0, None, 0)
        assert calls[-1][0] != ptr
    del cap
    eng.launch(0, None, 0)
    eng.launch(0, None, 0)
    assert ptr in [c[0] for c in calls[-2:]]

    class Owner:
        pass
    o = Owner()
    o.ob, o.tg = torch.zeros(10, 3, 2), torch.zeros(10, 1, 2)
    o.sn, o.tm = torch.zeros(10), torch.zeros(10, dtype=torch.bool)
    eng.track_state(torch.zeros(10, 3, 5), o.ob, o.tg, o.sn, o.tm, torch.zeros(10, 3, 5))
    cap = to_dlpack(eng.states())
    assert eng.shared_state()[0]
    del cap
    assert not eng.shared_state()[0]
    cap = to_dlpack(o.ob)
    assert eng.shared_state()[1]
    del cap
    assert not any(eng.shared_state())


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
