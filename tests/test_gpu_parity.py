"""Parity of the HIP step (libmarlnav.so through the drop-in Env) with the
reference's golden vectors and with the C oracle. Needs an MI355X."""
import os
import subprocess
import warnings

import numpy as np
import pytest
import torch

from conftest import (OBS_FIELDS, ROOT, RTOL, assert_obs_close, record_angle_stats,
                      record_threshold_stats,
                      assert_states_close, assert_vec_close, cli_args, env_values, golden, meta)

import oracle as orc

pytestmark = pytest.mark.gpu

STEP_CASES = ["step_a3o3", "step_a3o8", "step_a16o32", "step_a2o1", "step_p1"]
DEV = "cuda"


def np_(t):
    return t.detach().cpu().numpy()


def make_env(pkg, P, A, O, episode_len=200, rng="native", seed=1234, factors=None,
             sampler_num=-1, env_offset=0, **init_over):
    args = cli_args(num_parallel=P, num_agents=A, num_obstacles=O, episode_len=episode_len,
                    sampler_num=sampler_num, max_step=1000, **(factors or {}))
    params = pkg.set_env_params(args, DEV)
    params["init"] = dict(params["init"], **init_over)
    if params["sampler"] is not None:
        params["sampler"] = dict(params["sampler"])
    params["rng"] = rng
    params["seed"] = seed
    params["env_offset"] = env_offset
    return pkg.Env(params)


def fields_np(obs):
    return [np_(getattr(obs, f)) for f in OBS_FIELDS]


def oracle_params(env):
    env._sync_params()
    return env._dims, env._cparams


@pytest.mark.parametrize("name", STEP_CASES)
def test_step_matches_reference_golden(pkg, name):
    """F1 through the drop-in API, injecting state exactly as the golden
    generator injected it into the reference's Env."""
    m, z = meta(name), golden(name)
    P, A, O = m["num_parallel"], m["num_agents"], m["num_obstacles"]
    factors = {k: m[k] for k in ("risk_factor", "distance_factor", "heading_factor",
                                 "target_factor", "soft_factor", "bond_factor")}
    env = make_env(pkg, P, A, O, episode_len=m["episode_len"], rng="reference",
                   factors=factors, noise_device="cpu")
    for k in range(m["steps"]):
        env.states = torch.from_numpy(z["in_states"][k])
        env.obstacles = torch.from_numpy(z["in_obstacles"][k])
        env.target = torch.from_numpy(z["in_target"][k])
        env._step_num = torch.from_numpy(z["in_step_num"][k])
        env._terminates = torch.from_numpy(z["in_terminates"][k])
        fs, fo, ft = (torch.from_numpy(z[x][k]) for x in
                      ("fresh_states", "fresh_obstacles", "fresh_target"))
        env._init_sampler = lambda fs=fs, fo=fo, ft=ft: (fs, fo, ft)
        obs0 = env.observations()
        c0 = (env._num_trunc, env._num_col, env._num_tar)
        obs, rew, term, trunc = env.step(torch.from_numpy(z["actions"][k]).to(DEV))
        c1 = (env._num_trunc, env._num_col, env._num_tar)
        where = f"{name} step {k}"
        np.testing.assert_array_equal(np_(term), z["terminated"][k], where)
        np.testing.assert_array_equal(np_(trunc), z["truncated"][k], where)
        np.testing.assert_array_equal(np_(env._terminates), z["out_terminates"][k], where)
        np.testing.assert_array_equal(np_(env._step_num), z["out_step_num"][k], where)
        np.testing.assert_array_equal(np_(env.obstacles), z["out_obstacles"][k], where)
        np.testing.assert_array_equal(np_(env.target), z["out_target"][k], where)
        assert [b - a for a, b in zip(c0, c1)] == [z["d_trunc"][k], z["d_col"][k],
                                                     z["d_tar"][k]], where
        # rewards bit for bit (kernel = oracle bit for bit, and the oracle
        # reproduces every F1 reward, tests/test_oracle_golden.py)
        np.testing.assert_array_equal(np_(rew), z["reward"][k], where + " reward")
        assert_states_close(np_(env.states), z["out_states"][k], where)
        assert_obs_close(fields_np(obs), {f: z["obs_" + f][k] for f in OBS_FIELDS},
                         prefix="", where=where)
        record_angle_stats("golden F1", "reference", fields_np(obs),
                           [z["obs_" + f][k] for f in OBS_FIELDS])
        record_threshold_stats("golden F1 (kernel)", fields_np(obs))
        f0 = fields_np(obs0)
        for f, a in zip(OBS_FIELDS, f0):
            if "distance" in f:  # correctly rounded sqrt: bit-exact
                np.testing.assert_array_equal(a, z["obs0_" + f][k], where + " " + f)
        assert_obs_close(f0, {f: z["obs0_" + f][k] for f in OBS_FIELDS}, prefix="",
                         where=where + " observe")


@pytest.mark.parametrize("name", STEP_CASES)
def test_step_bit_exact_vs_oracle(pkg, name):
    """Same injected inputs through the oracle: every output bit for bit,
    bearings included (the oracle's acos is the kernel's, acos_device)."""
    m, z = meta(name), golden(name)
    P, A, O = m["num_parallel"], m["num_agents"], m["num_obstacles"]
    factors = {k: m[k] for k in ("risk_factor", "distance_factor", "heading_factor",
                                 "target_factor", "soft_factor", "bond_factor")}
    env = make_env(pkg, P, A, O, episode_len=m["episode_len"], rng="reference",
                   factors=factors, noise_device="cpu")
    dm, pr = oracle_params(env)
    for k in range(m["steps"]):
        ins = [z[x][k] for x in ("in_states", "in_obstacles", "in_target", "in_step_num",
                                 "in_terminates", "actions")]
        fresh = tuple(z[x][k] for x in ("fresh_states", "fresh_obstacles", "fresh_target"))
        exp = orc.step(dm, pr, *ins, fresh=fresh)
        env.states, env.obstacles, env.target = (torch.from_numpy(x) for x in ins[:3])
        env._step_num = torch.from_numpy(ins[3])
        env._terminates = torch.from_numpy(ins[4])
        env._init_sampler = lambda fs=fresh: tuple(torch.from_numpy(x) for x in fs)
        obs, rew, term, trunc = env.step(torch.from_numpy(ins[5]).to(DEV))
        where = f"{name} step {k}"
        np.testing.assert_array_equal(np_(env.states), exp["states"], where)
        np.testing.assert_array_equal(np_(rew), exp["reward"], where)
        np.testing.assert_array_equal(np_(term), exp["terminated"], where)
        np.testing.assert_array_equal(np_(trunc), exp["truncated"], where)
        got = np_(obs._packed)
        fo = orc.split_obs(exp["obs"], A, O)
        fg = orc.split_obs(got, A, O)
        for f, a, e in zip(OBS_FIELDS, fg, fo):
            if "distance" in f:
                np.testing.assert_array_equal(a, e, where + " " + f)
        assert_obs_close(fg, dict(zip(OBS_FIELDS, fo)), prefix="", exact=True, where=where)
        record_angle_stats("golden F1 inputs", "oracle", fg, fo)


def _trace_env(pkg, name):
    m = meta(name)
    args = cli_args(sampler_num=m["sampler_num"], max_step=m["steps"])
    if m["seed"] is not None:
        pkg.set_all_seeds(m["seed"])
    params = pkg.set_env_params(args, DEV)
    params["init"] = dict(params["init"], noise_device="cpu")
    params["rng"] = "reference"
    return m, pkg.Env(params)


@pytest.mark.parametrize("name", ["trace_cfg1", "trace_mock0", "trace_mock1"])
def test_trace_matches_reference(pkg, name):
    """F2/F3: the reward-check loop (utils.py:595-613) for 1000 steps through
    the drop-in Env, reference RNG mode: identical episodes and counters."""
    m, env = _trace_env(pkg, name)
    z = golden(name)
    np.testing.assert_array_equal(np_(env.states), z["states0"])
    np.testing.assert_array_equal(np_(env.obstacles), z["obstacles0"])
    A = env.num_agents
    O = env._dims.num_obstacles
    for k in range(m["steps"]):
        obs, rew, term, trunc = env.step(env.sample_actions())
        where = f"{name} step {k + 1}"
        np.testing.assert_array_equal(np_(term), z["terminated"][k], where)
        np.testing.assert_array_equal(np_(trunc), z["truncated"][k], where)
        np.testing.assert_array_equal(np_(env.obstacles), z["obstacles"][k], where)
        np.testing.assert_array_equal(np_(env.states), z["states"][k], where)
        np.testing.assert_array_equal(np_(rew), z["reward"][k], where + " reward")
        assert_obs_close(fields_np(obs), {f: z["obs_" + f][k] for f in OBS_FIELDS},
                         prefix="", where=where)
        record_angle_stats(f"trace {name}", "reference", fields_np(obs),
                           [z["obs_" + f][k] for f in OBS_FIELDS])
        record_threshold_stats(f"trace {name} (kernel)", fields_np(obs))
        if k % 100 == 99:
            assert (env._num_trunc, env._num_col, env._num_tar) == (
                z["num_trunc"][k], z["num_col"][k], z["num_tar"][k]), where
    assert (env._num_trunc, env._num_col, env._num_tar) == (
        z["num_trunc"][-1], z["num_col"][-1], z["num_tar"][-1])
    with pytest.raises(StopIteration) if m["sampler_num"] >= 0 else _nullctx():
        env.sample_actions()


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


@pytest.mark.parametrize("P,A,O,steps,ep", [(4096, 3, 3, 60, 25), (1000, 3, 8, 40, 25),
                                            (512, 16, 32, 12, 25), (333, 5, 2, 30, 25),
                                            (65536, 3, 3, 6, 25), (409600 + 27, 3, 3, 3, 25),
                                            (2 * 16384 * 32 + 5, 2, 1, 2, 25),
                                            (12000 + 7, 3, 3, 9, 4), (20480, 3, 8, 5, 2),
                                            (1021, 16, 32, 6, 3), (1000 + 3, 3, 8, 8, 3),
                                            (16384, 3, 3, 8, 3), (32768 + 5, 3, 3, 6, 4),
                                            (8192 + 3, 3, 3, 6, 2), (2048, 16, 32, 4, 2)])
def test_native_trajectory_bit_exact_vs_oracle(pkg, P, A, O, steps, ep):
    """Native (Philox) re-init mode, many steps, random actions, short
    episodes (ep = 2, 4: whole tiles finish at once, re-observed in several
    chunks): the GPU trajectory equals the oracle's bit for bit. The ragged
    split-kernel cases end on a workgroup with fewer live waves (1021 = 255*4
    + 1 one-env waves) and a partial tile (1003 envs, two per LPR-8 wave).
    16384 (configs[4]'s per-GPU shape), 8195 (ragged last block) and 32773
    envs at 3-step and shorter episodes: many finished envs every step.
    512, 1021 and 2048 x 16 x 32 run the split kernel's own-wave
    instantiation (finished envs re-initialised by their own wave)."""
    g = torch.Generator().manual_seed(P + A + O)
    env = make_env(pkg, P, A, O, episode_len=ep, seed=99,
                   factors=dict(risk_factor=3., distance_factor=7.))
    dm, pr = oracle_params(env)
    form = np_(env._formation)
    st, ob, tg = orc.reinit_all(dm, pr, form, 0)
    np.testing.assert_array_equal(np_(env.states), st)
    np.testing.assert_array_equal(np_(env.obstacles), ob)
    np.testing.assert_array_equal(np_(env.target), tg)
    sn = np.zeros(P, np.float32)
    te = np.zeros(P, np.bool_)
    tot = np.zeros(3, np.int64)
    for k in range(steps):
        th = (torch.rand(P, A, generator=g) - 0.5) * 0.8
        acc = (torch.rand(P, A, generator=g) - 0.5) * 1.2
        acts = torch.stack([th, acc], 2)
        exp = orc.step(dm, pr, st, ob, tg, sn, te, acts.numpy(), formation=form,
                       step_idx=k + 1)
        obs, rew, term, trunc = env.step(acts.to(DEV))
        where = f"P{P} A{A} O{O} step {k + 1}"
        np.testing.assert_array_equal(np_(env.states), exp["states"], where)
        np.testing.assert_array_equal(np_(env.obstacles), exp["obstacles"], where)
        np.testing.assert_array_equal(np_(env.target), exp["target"], where)
        np.testing.assert_array_equal(np_(env._step_num), exp["step_num"], where)
        np.testing.assert_array_equal(np_(env._terminates), exp["terminates"], where)
        np.testing.assert_array_equal(np_(term), exp["terminated"], where)
        np.testing.assert_array_equal(np_(trunc), exp["truncated"], where)
        np.testing.assert_array_equal(np_(rew), exp["reward"], where)
        got = np_(obs._packed)
        Oe = dm.num_obstacles
        fg, fo = orc.split_obs(got, A, Oe), orc.split_obs(exp["obs"], A, Oe)
        assert_obs_close(fg, dict(zip(OBS_FIELDS, fo)), prefix="", exact=True, where=where)
        st, ob, tg, sn, te = (exp[x] for x in ("states", "obstacles", "target", "step_num",
                                               "terminates"))
        tot += exp["counters"]
    assert [env._num_trunc, env._num_col, env._num_tar] == tot.tolist()
    assert (tot[1] > 0 or steps < 10) and (tot[0] > 0 or steps < ep)  # terminal paths hit


@pytest.mark.parametrize("P,A,O,template", [(1000 + 3, 3, 8, False), (2048 + 5, 3, 8, False),
                                            (1000 + 3, 3, 8, True)])
def test_native_a3o8_finished_env_paths_bit_exact_vs_oracle(pkg, P, A, O, template):
    """The split kernel's A3/O8 finished envs (native re-init, two-step
    episodes: every env finishes every other step) through the workgroup-wide
    fused re-init pass, with the formation template passed and without it (a
    C-ABI caller that passes no formation_obs), at LPR 8 (1003 envs, a
    partial last tile) and LPR 4 (2053 envs). (Round 6 also ran this against
    the speculative fresh-row variant, MARLNAV_SPLIT_SPEC at eb3feb8, which
    took the template path.)"""
    g = torch.Generator().manual_seed(P + 17 * template)
    env = make_env(pkg, P, A, O, episode_len=2, seed=7)
    if not template:
        env._formation_obs = None
        env._configure()
    dm, pr = oracle_params(env)
    form = np_(env._formation)
    st, ob, tg = orc.reinit_all(dm, pr, form, 0)
    sn = np.zeros(P, np.float32)
    te = np.zeros(P, np.bool_)
    n_fin = 0
    for k in range(6):
        acts = torch.stack([(torch.rand(P, A, generator=g) - 0.5) * 0.8,
                            (torch.rand(P, A, generator=g) - 0.5) * 1.2], 2)
        exp = orc.step(dm, pr, st, ob, tg, sn, te, acts.numpy(), formation=form, step_idx=k + 1)
        obs, rew, term, trunc = env.step(acts.to(DEV))
        where = f"P{P} template={template} step {k + 1}"
        for got, key in ((env.states, "states"), (env.obstacles, "obstacles"),
                         (env.target, "target"), (rew, "reward"), (term, "terminated"),
                         (trunc, "truncated")):
            np.testing.assert_array_equal(np_(got), exp[key], where + " " + key)
        fg, fo = orc.split_obs(np_(obs._packed), A, O), orc.split_obs(exp["obs"], A, O)
        assert_obs_close(fg, dict(zip(OBS_FIELDS, fo)), prefix="", exact=True, where=where)
        st, ob, tg, sn, te = (exp[x] for x in ("states", "obstacles", "target", "step_num",
                                               "terminates"))
        n_fin += int((exp["step_num"] == 0.0).sum())
    assert n_fin > 0  # the finished-env paths ran


def test_threshold_proximity_native_65536(pkg):
    """on the headline workload (65 536 x 3 x 3, native
    re-init, random turns, 100 steps) count the observation entries within
    4 ulp of a reward / terminal threshold (printed in the summary). Those
    are the only entries whose flag could differ from the reference's when
    a bearing or distance is 1-2 ulp away from it; the kernel equals the
    oracle on all of them (test_native_trajectory_bit_exact_vs_oracle)."""
    P, A, O = 65536, 3, 3
    g = torch.Generator().manual_seed(2025)
    env = make_env(pkg, P, A, O, episode_len=200, seed=4242)
    for k in range(100):
        th = (torch.rand(P, A, generator=g) - 0.5) * 0.8
        acc = (torch.rand(P, A, generator=g) - 0.5) * 1.2
        obs, rew, term, trunc = env.step(torch.stack([th, acc], 2).to(DEV))
        if k % 10 == 9:  # every 10th step: 10 x 196 608 rows
            record_threshold_stats("native 65536x3x3 (kernel, 10 of 100 steps)", fields_np(obs))
    assert np.isfinite(np_(rew)).all()


def test_counters_reset_like_mappo(pkg):
    """MAPPO reads then assigns 0 to the counters (models.py:151-158)."""
    env = make_env(pkg, 2048, 3, 3, episode_len=5)
    for _ in range(12):
        env.step(torch.zeros(2048, 3, 2, device=DEV))
    assert env._num_trunc >= 2048
    env._num_trunc = 0
    env._num_col = 0
    env._num_tar = 7
    assert (env._num_trunc, env._num_col, env._num_tar) == (0, 0, 7)
    env.step(torch.zeros(2048, 3, 2, device=DEV))
    assert env._num_trunc == 0 and env._num_tar == 7


def test_fused_normalizer_and_action_scaler(pkg):
    """§8(f) rows 1-2: ObsNormalizer fused into the step equals the host
    normalizer (utils.py:519-532) on the returned obs; ActionScaler
    (utils.py:535-547) applied outside gives the same step."""
    args = cli_args(num_parallel=3000, num_obstacles=3)
    nrm = pkg.ObsNormalizer(pkg.set_normalizer_params(args, DEV))
    scl = pkg.ActionScaler(pkg.set_scaler_params(args, DEV))
    env = make_env(pkg, 3000, 3, 3, episode_len=15)
    env.attach_normalizer(nrm)
    g = torch.Generator().manual_seed(5)
    for _ in range(20):
        raw = (torch.rand(3000, 3, 2, generator=g) * 2 - 1).to(DEV)
        obs, rew, term, trunc = env.step(scl(raw))
        fused = nrm(obs)
        ref = (torch.cat(tuple(obs), dim=2) - nrm.mean) / nrm.scale_tensor
        assert fused is obs._normalized
        torch.testing.assert_close(fused, ref, rtol=0, atol=0)


def test_fused_action_scaler(pkg):
    """§8(f) row 2: an attached ActionScaler (utils.py:535-547) applied in the
    kernel's action load equals scaling on the host first, bit for bit."""
    args = cli_args(num_parallel=2000, num_obstacles=3)
    scl = pkg.ActionScaler(pkg.set_scaler_params(args, DEV))
    fused = make_env(pkg, 2000, 3, 3, episode_len=12)
    plain = make_env(pkg, 2000, 3, 3, episode_len=12)
    fused.attach_action_scaler(scl)
    g = torch.Generator().manual_seed(11)
    for k in range(25):
        raw = (torch.rand(2000, 3, 2, generator=g) * 2 - 1).to(DEV)
        o1, r1, te1, tr1 = fused.step(raw)
        o2, r2, te2, tr2 = plain.step(scl(raw))
        assert torch.equal(fused.states, plain.states), k
        assert torch.equal(r1, r2) and torch.equal(te1, te2) and torch.equal(tr1, tr2), k
        assert torch.equal(o1._packed, o2._packed), k
    fused.attach_action_scaler(None)
    raw = torch.rand(2000, 3, 2, generator=g).to(DEV)
    fused.step(raw)
    plain.step(raw)
    assert torch.equal(fused.states, plain.states)


def test_observations_reset_and_api(pkg):
    env = make_env(pkg, 10, 3, 3)
    obs, params = env.reset()
    assert params is env.params
    assert isinstance(obs, pkg.Observations)
    assert [tuple(x.shape) for x in obs] == [(10, 3, 1), (10, 3, 1), (10, 3, 3), (10, 3, 3),
                                            (10, 3, 2), (10, 3, 2)]
    assert torch.equal(env._reinit_mask, torch.ones(10, device=DEV))
    o2, r, te, tr = env.step(env.sample_actions())
    assert r.shape == (10,) and r.dtype == torch.float32
    assert te.dtype == torch.bool and tr.dtype == torch.bool
    assert env._reinit_mask.dtype == torch.int64
    # non-contiguous / wider actions are accepted like the reference's slicing
    wide = torch.zeros(10, 3, 4, device=DEV)
    env.step(wide)
    with pytest.raises(ValueError):
        env.step(torch.zeros(9, 3, 2, device=DEV))


def test_sharded_native_init_is_invariant(pkg):
    """Philox keyed on the global env id: two shards == one whole batch."""
    full = make_env(pkg, 1000, 3, 3, seed=7)
    a = make_env(pkg, 400, 3, 3, seed=7, env_offset=0)
    b = make_env(pkg, 600, 3, 3, seed=7, env_offset=400)
    torch.testing.assert_close(full.obstacles, torch.cat([a.obstacles, b.obstacles]),
                               rtol=0, atol=0)
    acts = torch.zeros(1000, 3, 2, device=DEV)
    acts[:, :, 1] = 0.5
    for _ in range(30):
        full.step(acts)
        a.step(acts[:400])
        b.step(acts[400:])
    torch.testing.assert_close(full.states, torch.cat([a.states, b.states]), rtol=0, atol=0)
    torch.testing.assert_close(full.obstacles, torch.cat([a.obstacles, b.obstacles]),
                               rtol=0, atol=0)


def test_step_outputs_never_alias_live_tensors(pkg):
    """Env.step recycles output memory only when nothing refers to it: kept
    outputs, kept views and kept Observations tuples are never overwritten."""
    env = make_env(pkg, 777, 3, 3, episode_len=9)
    acts = [torch.rand(777, 3, 2, device=DEV) - 0.5 for _ in range(4)]
    kept = []
    for k in range(12):
        obs, rew, term, trunc = env.step(acts[k % 4])
        if k % 3 == 0:
            kept.append(("obs", obs, obs._packed.clone()))
        elif k % 3 == 1:
            kept.append(("view", obs.obstacles_distances[5:9], obs.obstacles_distances[5:9].clone()))
            kept.append(("rew", rew, rew.clone()))
        else:
            kept.append(("term", term, term.clone()))
            kept.append(("trunc", trunc, trunc.clone()))
        del obs, rew, term, trunc
    torch.cuda.synchronize()
    for what, live, snap in kept:
        cur = live._packed if what == "obs" else live
        assert torch.equal(cur, snap), what
    # nothing kept: the memory is recycled (bounded pool)
    ptrs = set()
    for k in range(10):
        o, r, te, tr = env.step(acts[k % 4])
        ptrs.add(o._packed.data_ptr())
        del o, r, te, tr
    assert len(ptrs) <= 4


def test_held_state_tensors_see_what_the_reference_shows(pkg):
    """The reference never writes obstacles / target in place (its re-init
    rebinds them, environment.py:79-81): a caller holding the pre-step tensor,
    or a view of it, keeps its values here too. A held `states` receives the
    moved states (the reference moves in place, :113-123) but not the re-init
    (:79 rebinds). Nothing held: the step writes the Env's buffers in place (no
    copies). Holders change nothing else: the trajectory equals one run
    without holders, bit for bit."""
    P = 4096 + 7
    env = make_env(pkg, P, 3, 3, episode_len=3)   # every env truncates at step 3
    twin = make_env(pkg, P, 3, 3, episode_len=3)
    acts = [torch.rand(P, 3, 2, device=DEV) - 0.5 for _ in range(3)]
    p_st, p_ob, p_tg = env.states.data_ptr(), env.obstacles.data_ptr(), env.target.data_ptr()
    for k in range(4):
        env.step(acts[k % 3])
        twin.step(acts[k % 3])
    assert (env.states.data_ptr(), env.obstacles.data_ptr(), env.target.data_ptr()) == \
        (p_st, p_ob, p_tg)
    ob, tg_view = env.obstacles, env.target[:, 0]
    ob0, tg0 = ob.clone(), tg_view.clone()
    for k in range(4, 8):
        if k == 5:   # step 6: every env truncates
            held, held0 = env.states, env.states.clone()
            ob_k, tg_k = env.obstacles.clone(), env.target.clone()
        o1 = env.step(acts[k % 3])[0]
        o2 = twin.step(acts[k % 3])[0]
        assert torch.equal(o1._packed, o2._packed)
        if k == 5:
            # the moved states alone: the same pre-step state through an Env
            # in which nothing finishes
            mv = make_env(pkg, P, 3, 3, episode_len=10 ** 9)
            mv._ob_coll_dist = mv._ag_coll_dist = float("-inf")
            mv.states, mv.obstacles, mv.target = held0, ob_k, tg_k
            mv.step(acts[k % 3])
            torch.cuda.synchronize()
            assert torch.equal(held, mv.states)
            assert not torch.equal(held, env.states)   # the env's own: re-initialised
            del held, mv
    torch.cuda.synchronize()
    assert torch.equal(ob, ob0) and torch.equal(tg_view, tg0)
    assert env.obstacles.data_ptr() != p_ob and env.target.data_ptr() != p_tg
    assert not torch.equal(env.obstacles, ob0)    # its own buffer was re-initialised
    for a, b in ((env.states, twin.states), (env.obstacles, twin.obstacles),
                 (env.target, twin.target)):
        assert torch.equal(a, b)
    # holders gone (the loop's names too): back to in-place steps
    del ob, tg_view, a, b
    q = (env.states.data_ptr(), env.obstacles.data_ptr(), env.target.data_ptr())
    for k in range(3):
        env.step(acts[k])
    assert (env.states.data_ptr(), env.obstacles.data_ptr(), env.target.data_ptr()) == q


def test_held_states_reference_rng_mode(pkg):
    """The same held-`states` rule through Env._step_py's reference-RNG
    branch (host-drawn fresh candidates every step, environment.py:78)."""
    P = 3000 + 5
    env = make_env(pkg, P, 3, 3, episode_len=2, rng="reference")
    acts = torch.rand(P, 3, 2, device=DEV) - 0.5
    env.step(acts)
    held, held0 = env.states, env.states.clone()
    ob_k, tg_k = env.obstacles.clone(), env.target.clone()
    env.step(acts)                      # step 2: every env truncates
    mv = make_env(pkg, P, 3, 3, episode_len=10 ** 9)
    mv._ob_coll_dist = mv._ag_coll_dist = float("-inf")
    mv.states, mv.obstacles, mv.target = held0, ob_k, tg_k
    mv.step(acts)
    torch.cuda.synchronize()
    assert torch.equal(held, mv.states)
    assert not torch.equal(held, env.states)


@pytest.mark.parametrize("P,A,O", [(4096 + 5, 3, 3), (60, 16, 32), (333, 5, 2)])
def test_double_buffered_states(pkg, P, A, O):
    """params['states_double_buffer'] (MarlnavStepBuffers.states_out): the
    step reads one state buffer and writes the other, the two alternating
    with no allocation; every output and state bit-identical to the in-place
    Env, a held `states` still sees what the reference shows (the moved
    states), and the buffer it holds is replaced, not written, afterwards."""
    env = make_env(pkg, P, A, O, episode_len=4)
    params = dict(env.params, states_double_buffer=True)
    db2 = pkg.Env(params)
    acts = [torch.rand(P, A, 2, device=DEV) - 0.5 for _ in range(3)]
    ptrs = set()
    for k in range(9):
        o1, r1, te1, tr1 = env.step(acts[k % 3])
        o2, r2, te2, tr2 = db2.step(acts[k % 3])
        ptrs.add(db2.states.data_ptr())
        assert torch.equal(o1._packed, o2._packed) and torch.equal(r1, r2)
        assert torch.equal(te1, te2) and torch.equal(tr1, tr2)
        assert torch.equal(env.states, db2.states)
        if k == 5:
            held, held0 = db2.states, db2.states.clone()
            ob_k, tg_k = db2.obstacles.clone(), db2.target.clone()
        if k == 6:
            mv = make_env(pkg, P, A, O, episode_len=10 ** 9)
            mv._ob_coll_dist = mv._ag_coll_dist = float("-inf")
            mv.states, mv.obstacles, mv.target = held0, ob_k, tg_k
            mv.step(acts[k % 3])
            torch.cuda.synchronize()
            assert torch.equal(held, mv.states)
            moved = held.clone()
            del mv
        if k == 8:
            torch.cuda.synchronize()
            assert torch.equal(held, moved)   # not written by later steps
    assert len(ptrs) >= 2 and all(p != held.data_ptr() for p in [db2.states.data_ptr()])
    # the host swaps the two buffers once per call: a captured step would
    # replay reading one buffer and writing the other forever, so capture is
    # refused even with allow_graph_capture
    db2.allow_graph_capture = True
    graph = torch.cuda.CUDAGraph()
    scratch = torch.zeros(1, device=DEV)
    with pytest.raises(RuntimeError, match="double-buffered"):
        with torch.cuda.graph(graph):
            scratch += 1   # (a non-empty capture whatever the step does)
            db2.step(acts[0])
    torch.cuda.synchronize()


def test_held_states_pair_split_kernel(pkg):
    """The held-`states` rule on the pair-split kernel family (A16/O32, the
    configs[3] shape; test_held_state_tensors_see_what_the_reference_shows
    covers the env-block kernel): a held pre-step `states` receives the
    moved states of a step in which every env truncates, the Env's own
    tensor the re-initialised ones."""
    P, A, O = 60, 16, 32
    env = make_env(pkg, P, A, O, episode_len=2)
    acts = torch.rand(P, A, 2, device=DEV) - 0.5
    env.step(acts)
    assert env._lib.marlnav_debug_last_family() == 2   # MARLNAV_FAMILY_SPLIT
    held, held0 = env.states, env.states.clone()
    ob_k, tg_k = env.obstacles.clone(), env.target.clone()
    env.step(acts)                      # step 2: every env truncates
    mv = make_env(pkg, P, A, O, episode_len=10 ** 9)
    mv._ob_coll_dist = mv._ag_coll_dist = float("-inf")
    mv.states, mv.obstacles, mv.target = held0, ob_k, tg_k
    mv.step(acts)
    torch.cuda.synchronize()
    assert torch.equal(held, mv.states)
    assert not torch.equal(held, env.states)


def test_held_step_num_and_terminates_see_what_the_reference_shows(pkg):
    """`_step_num` is incremented in place (environment.py:96) and then
    rebound by the re-init (:83); `_terminates` is rebound at :219. A caller
    holding either from before a step sees the reference's: step_num + 1 for
    every env (finished ones included), the old terminates flags; the Env's
    own tensors carry on as in a run without holders."""
    P = 4096 + 3
    env = make_env(pkg, P, 3, 3, episode_len=3)
    twin = make_env(pkg, P, 3, 3, episode_len=3)
    acts = [torch.rand(P, 3, 2, device=DEV) - 0.5 for _ in range(3)]
    for k in range(2):
        env.step(acts[k])
        twin.step(acts[k])
    sn, tm = env._step_num, env._terminates
    sn0, tm0 = sn.clone(), tm.clone()
    env.step(acts[2])                   # step 3: every env truncates
    twin.step(acts[2])
    torch.cuda.synchronize()
    assert torch.equal(sn, sn0 + 1.0) and torch.equal(tm, tm0)
    assert torch.equal(env._step_num, twin._step_num)
    assert torch.equal(env._terminates, twin._terminates)
    assert float(env._step_num.max()) == 0.0        # re-initialised: rebound to zeros
    assert torch.equal(env.states, twin.states)


def test_reinit_mask_survives_state_assignment(pkg):
    """`_reinit_mask` (environment.py:102-103) is the last step's
    where(truncated | terminated, 1, 0) even after an assignment that drops
    the engine's output sets (states, obstacles, target, a normaliser)."""
    P = 300
    env = make_env(pkg, P, 3, 3, episode_len=2)
    acts = torch.rand(P, 3, 2, device=DEV) - 0.5
    env.step(acts)
    _, _, term, trunc = env.step(acts)       # step 2: every env truncates
    want = torch.where(torch.logical_or(trunc, term), 1, 0)
    del term, trunc
    env.states = env.states.clone()
    assert torch.equal(env._reinit_mask, want)
    env.obstacles = env.obstacles.clone()
    assert torch.equal(env._reinit_mask, want) and int(want.sum()) == P


def test_subclass_step_override_is_called(pkg):
    """A subclass overriding step keeps its method (the engine binds itself
    on the instance only for Env's own step) and reaches the native step
    through super().step."""
    base = pkg.Env

    class Scaled(base):
        calls = 0

        def step(self, actions):
            Scaled.calls += 1
            obs, rew, term, trunc = super().step(actions)
            return obs, rew * 2.0, term, trunc

    P = 200
    args = cli_args(num_parallel=P, episode_len=50)
    params = pkg.set_env_params(args, DEV)
    params.update(rng="native", seed=7)
    sub, ref = Scaled(params), base(params)
    acts = torch.rand(P, 3, 2, device=DEV) - 0.5
    for _ in range(3):
        _, r1, _, _ = sub.step(acts)
        _, r0, _, _ = ref.step(acts)
        assert torch.equal(r1, r0 * 2.0)
    assert Scaled.calls == 3
    assert "step" not in sub.__dict__ and "step" in ref.__dict__


def test_discounted_returns_match_reference_and_oracle(pkg):
    """§8(f) row 3: the device scan against MAPPO._process_rewards run
    unmodified (F5) and the C oracle at rollout size; float64 within 1e-12."""
    from conftest import golden, meta
    z = golden("process_rewards")
    for k, m in enumerate(meta("process_rewards")["cases"]):
        rew = torch.from_numpy(z[f"case{k}_rewards"]).to(DEV)
        done = torch.from_numpy(z[f"case{k}_done"]).to(DEV)
        ret, mean, std = pkg.rollout.discounted_returns(rew, done, m["gamma"])
        np.testing.assert_allclose(np_(ret), z[f"case{k}_returns"], rtol=1e-12, atol=1e-12)
        assert abs(mean.item() - float(z[f"case{k}_mean"])) <= 1e-12 * max(1., abs(mean.item()))
    g = torch.Generator().manual_seed(3)
    T, P = 64, 65536 + 17
    rew = torch.randn(T, P, generator=g) * 50
    done = torch.rand(T, P, generator=g) < 0.02
    ret, mean, std = pkg.rollout.discounted_returns(rew.to(DEV), done.to(DEV), 0.97)
    oret, (omean, ostd) = orc.discounted_returns(rew.numpy(), done.numpy(), 0.97)
    np.testing.assert_allclose(np_(ret), oret, rtol=1e-10, atol=1e-10)
    assert abs(mean.item() - omean) <= 1e-12 * abs(omean) and abs(std.item() - ostd) <= 1e-12 * ostd


def test_process_rewards_list_buffer_and_rollout_buffer(pkg):
    """The list-buffer drop-in updates entries like models.py:134-144; the
    stacked RolloutBuffer gives the same returns."""
    from conftest import golden, meta
    z = golden("process_rewards")
    m = meta("process_rewards")["cases"][0]
    rew = torch.from_numpy(z["case0_rewards"]).to(DEV)
    done = torch.from_numpy(z["case0_done"]).to(DEV)
    T, P = rew.shape
    obs = torch.zeros(P, 3, 12, device=DEV)
    buf = [[obs, None, None, None, rew[t].clone(), done[t].clone()] for t in range(T)]
    mean = pkg.rollout.process_rewards(buf, m["gamma"])
    assert buf[0][0] is obs and buf[0][-2].dtype == torch.float64
    np.testing.assert_allclose(np.stack([np_(e[-2]) for e in buf]), z["case0_returns"],
                               rtol=1e-12, atol=1e-12)
    rb = pkg.rollout.RolloutBuffer(T)
    for t in range(T):
        rb.add(obs, torch.zeros(P * 3, 2, device=DEV), torch.zeros(P * 3, device=DEV),
               torch.zeros(P, 1, device=DEV), rew[t], done[t])
    mean2 = rb.process_rewards(m["gamma"])
    assert mean2.item() == mean.item()
    ents = rb.entries()
    assert len(ents) == T and ents[3][4].dtype == torch.float64
    np.testing.assert_array_equal(np.stack([np_(e[4]) for e in ents]),
                                  np.stack([np_(e[-2]) for e in buf]))


def _check_rews_expected(z, steps, p, a, A=3, O=3):
    """The nine check_rews series (utils.py:595-613) read off a trace fixture."""
    return {
        "target_angles": z["obs_target_angle"][:steps, p, a, 0],
        "target_distances": z["obs_target_distance"][:steps, p, a, 0],
        "all_obs_angels": z["obs_obstacles_angles"][:steps, p, a, 0],
        "all_obs_distances": z["obs_obstacles_distances"][:steps, p, a, 0],
        "angles_to_first": z["obs_others_angles"][:steps, p, a, 0],
        "distances_to_first": z["obs_others_distances"][:steps, p, a, 0],
        "angles_to_second": z["obs_others_angles"][:steps, p, a, 1],
        "distances_to_second": z["obs_others_distances"][:steps, p, a, 1],
        "rewards": z["reward"][:steps, p],
    }


@pytest.mark.parametrize("name,agent", [("trace_cfg1", 0), ("trace_mock1", 2)])
def test_check_rews_series_match_reference(pkg, name, agent, tmp_path):
    """§8(f) row 4: check_rews (utils.py:579-666) records the reference's nine
    series (F2/F3 traces) and writes its two figures."""
    m, env = _trace_env(pkg, name)
    z = golden(name)
    steps = 300
    series = pkg.utils.check_rews(env, steps, 1, agent, plot_dir=str(tmp_path), plot=True)
    exp = _check_rews_expected(z, steps, 1, agent, O=z["obs_obstacles_angles"].shape[-1])
    assert list(series) == list(pkg.utils.CHECK_REWS_SERIES)
    for k, v in exp.items():
        atol = 0.0
        np.testing.assert_allclose(np.asarray(series[k]), v, rtol=RTOL, atol=atol, err_msg=k)
    names = sorted(os.listdir(tmp_path))
    assert f"states_array_1_agent_{agent}.png" in names and any(n.startswith("rewards_B1") for n in names)


def test_cli_reward_check_matches_reference(pkg):
    """``python -m marlnav_amd -rc -se 0 --init-noise-device cpu`` prints the
    reference's CPU config-1 series (F2) - the plumbing run of BASELINE
    configs[0]."""
    import subprocess
    import sys
    steps = 120
    out = subprocess.run([sys.executable, "-m", "marlnav_amd", "-rc", "-se", "0", "-ms", str(steps),
                          "--no-plots", "--init-noise-device", "cpu"], cwd=ROOT,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    got = {}
    for line in out.stdout.splitlines():
        k, *vals = line.split()
        got[k] = np.array([float(v) for v in vals])
    exp = _check_rews_expected(golden("trace_cfg1"), steps, 0, 0)
    for k, v in exp.items():
        atol = 0.0
        np.testing.assert_allclose(got[k], v, rtol=2e-8 + RTOL, atol=atol + 1e-7, err_msg=k)


@pytest.mark.parametrize("P,A,O", [(16384, 3, 3), (20480, 3, 8), (4096, 3, 3), (1024, 3, 8),
                                   (512, 16, 32)])
def test_extreme_coordinates_take_the_exact_path(pkg, P, A, O):
    """Tiles holding coordinates outside the fast pair math's range (tiny,
    huge, coincident points) fall back to IEEE sqrt/division for the whole
    wave; every env still equals the oracle bit for bit."""
    g = torch.Generator().manual_seed(O + A)
    env = make_env(pkg, P, A, O, episode_len=9, seed=5)
    st = env.states.cpu().clone()
    ob = env.obstacles.cpu().clone()
    tg = env.target.cpu().clone()
    st[5, 1, :2] = torch.tensor([1e-25, 3e-30])          # tiny positions
    st[6, 0, :2] = torch.tensor([2e-39, 0.0])            # subnormal
    st[7, 2, :2] = st[7, 0, :2]                          # coincident agents
    ob[40, 0] = torch.tensor([1e30, 5.0])                # huge obstacle
    tg[100, 0] = torch.tensor([0.0, 1e-22])
    st[300, 1, :2] = torch.tensor([3e12, -7e11])          # beyond 2^40
    env.states, env.obstacles, env.target = st, ob, tg
    dm, pr = oracle_params(env)
    form = np_(env._formation)
    s, o, t = st.numpy(), ob.numpy(), tg.numpy()
    sn = np.zeros(P, np.float32)
    te = np.zeros(P, np.bool_)
    for k in range(3):
        acts = (torch.rand(P, A, 2, generator=g) - 0.5)
        exp = orc.step(dm, pr, s, o, t, sn, te, acts.numpy(), formation=form, step_idx=k + 1)
        obs, rew, term, trunc = env.step(acts.to(DEV))
        where = f"P{P} A{A} O{O} step {k + 1}"
        np.testing.assert_array_equal(np_(env.states), exp["states"], where)
        np.testing.assert_array_equal(np_(rew), exp["reward"], where)
        np.testing.assert_array_equal(np_(term), exp["terminated"], where)
        got = np_(obs._packed)
        np.testing.assert_array_equal(got[..., 1], exp["obs"][..., 1], where)  # distances exact
        fg, fo = orc.split_obs(got, A, O), orc.split_obs(exp["obs"], A, O)
        assert_obs_close(fg, dict(zip(OBS_FIELDS, fo)), prefix="", exact=True, where=where)
        s, o, t, sn, te = (exp[x] for x in ("states", "obstacles", "target", "step_num",
                                            "terminates"))


@pytest.mark.parametrize("P,A,O", [(20000 + 13, 3, 3), (8192 + 5, 3, 8), (300, 3, 3), (60, 3, 3)])
def test_reference_rng_fresh_candidates_bit_exact_vs_oracle(pkg, P, A, O):
    """rng='reference' at block-kernel sizes (and one split-kernel size):
    finished envs take the host's fresh candidates (environment.py:76-90
    with the sampler call at :78); episodes of 3 steps so whole blocks finish
    together; the last block is ragged. Bit-exact vs the oracle."""
    g = torch.Generator().manual_seed(P * 7 + O)
    env = make_env(pkg, P, A, O, episode_len=3, rng="reference", noise_device="cpu",
                   factors=dict(risk_factor=2., bond_factor=5.))
    dm, pr = oracle_params(env)
    st, ob, tg = (np_(x).copy() for x in (env.states, env.obstacles, env.target))
    sn = np.zeros(P, np.float32)
    te = np.zeros(P, np.bool_)
    tot = np.zeros(3, np.int64)
    for k in range(7):
        fs = (torch.rand(P, A, 5, generator=g) * 900.0).numpy()
        fo = (torch.rand(P, O, 2, generator=g) * 700.0).numpy()
        ft = (torch.rand(P, 1, 2, generator=g) * 1400.0).numpy()
        fresh = (fs, fo, ft)
        env._init_sampler = lambda fr=fresh: tuple(torch.from_numpy(x) for x in fr)
        acts = ((torch.rand(P, A, 2, generator=g) - 0.5) * 0.9).numpy()
        exp = orc.step(dm, pr, st, ob, tg, sn, te, acts, fresh=fresh)
        obs, rew, term, trunc = env.step(torch.from_numpy(acts).to(DEV))
        where = f"P{P} A{A} O{O} step {k + 1}"
        for name, got in (("states", env.states), ("obstacles", env.obstacles),
                          ("target", env.target), ("step_num", env._step_num),
                          ("terminates", env._terminates), ("terminated", term),
                          ("truncated", trunc), ("reward", rew)):
            np.testing.assert_array_equal(np_(got), exp[name], where + " " + name)
        fg, fo_ = orc.split_obs(np_(obs._packed), A, O), orc.split_obs(exp["obs"], A, O)
        assert_obs_close(fg, dict(zip(OBS_FIELDS, fo_)), prefix="", exact=True, where=where)
        st, ob, tg, sn, te = (exp[x] for x in ("states", "obstacles", "target", "step_num",
                                               "terminates"))
        tot += exp["counters"].astype(np.int64)
    assert tot[0] >= P  # every env truncated at least once
    assert [env._num_trunc, env._num_col, env._num_tar] == tot.tolist()


@pytest.mark.parametrize("P,A,O", [(16384 + 9, 3, 3), (1000, 3, 8), (512, 16, 32)])
def test_native_noisy_agents_bit_exact_vs_oracle(pkg, P, A, O):
    """Native re-init with noisy agent positions and headings
    (TriangleIntitializer noisy_ags, utils.py:350-368): the NOISY kernel
    instantiations (block, split and generic) equal the oracle bit for bit."""
    g = torch.Generator().manual_seed(P + 11 * O)
    env = make_env(pkg, P, A, O, episode_len=3, seed=7, noisy_ags=True)
    dm, pr = oracle_params(env)
    form = np_(env._formation)
    st, ob, tg = orc.reinit_all(dm, pr, form, 0)
    np.testing.assert_array_equal(np_(env.states), st)
    sn = np.zeros(P, np.float32)
    te = np.zeros(P, np.bool_)
    for k in range(5):
        acts = ((torch.rand(P, A, 2, generator=g) - 0.5) * 0.8).numpy()
        exp = orc.step(dm, pr, st, ob, tg, sn, te, acts, formation=form, step_idx=k + 1)
        obs, rew, term, trunc = env.step(torch.from_numpy(acts).to(DEV))
        where = f"P{P} A{A} O{O} step {k + 1}"
        for name, got in (("states", env.states), ("obstacles", env.obstacles),
                          ("target", env.target), ("step_num", env._step_num),
                          ("reward", rew), ("terminated", term)):
            np.testing.assert_array_equal(np_(got), exp[name], where + " " + name)
        fg, fo_ = orc.split_obs(np_(obs._packed), A, O), orc.split_obs(exp["obs"], A, O)
        assert_obs_close(fg, dict(zip(OBS_FIELDS, fo_)), prefix="", exact=True, where=where)
        st, ob, tg, sn, te = (exp[x] for x in ("states", "obstacles", "target", "step_num",
                                               "terminates"))


FAMILIES = {1: "block", 2: "split", 4: "wave"}


@pytest.mark.parametrize("P,A,O,expect", [
    (4096 + 5, 3, 3, {1, 2, 4}),      # every family holds the A3/O3 shape
    (2048 + 3, 3, 8, {1, 2, 4}),
    (5000 + 1, 2, 1, {1, 4}),         # no split variant at A2/O1
    (200, 16, 32, {2, 4}),            # split (compiled) or the generic wave kernel
    (777, 5, 2, {4}),                 # runtime shape: wave kernel only
])
def test_every_kernel_family_bit_exact_vs_oracle(pkg, P, A, O, expect):
    """The host picks one of three kernel families by shape and grid size
    (DESIGN.md §3); the automatic choice leaves some of them unused at the
    sizes above. Force each in turn (marlnav_debug_force_family) over the
    same seeded trajectory - native re-init, 3-step episodes, the observe-only
    instantiation through Env.observations() - and check each against the
    oracle bit for bit."""
    ran = set()
    for fam in FAMILIES:
        g = torch.Generator().manual_seed(P + A + O)
        env = make_env(pkg, P, A, O, episode_len=3, seed=21,
                       factors=dict(risk_factor=3., distance_factor=7., bond_factor=2.))
        lib = env._lib
        prev = lib.marlnav_debug_force_family(fam)
        try:
            dm, pr = oracle_params(env)
            form = np_(env._formation)
            st, ob, tg = orc.reinit_all(dm, pr, form, 0)
            sn = np.zeros(P, np.float32)
            te = np.zeros(P, np.bool_)
            for k in range(4):
                acts = ((torch.rand(P, A, 2, generator=g) - 0.5) * 0.8).numpy()
                exp = orc.step(dm, pr, st, ob, tg, sn, te, acts, formation=form,
                               step_idx=k + 1)
                obs, rew, term, trunc = env.step(torch.from_numpy(acts).to(DEV))
                torch.cuda.synchronize()
                got_fam = lib.marlnav_debug_last_family()
                where = f"P{P} A{A} O{O} forced {FAMILIES[fam]} ran {FAMILIES[got_fam]} step {k + 1}"
                for name, got in (("states", env.states), ("obstacles", env.obstacles),
                                  ("target", env.target), ("step_num", env._step_num),
                                  ("terminates", env._terminates), ("reward", rew),
                                  ("terminated", term), ("truncated", trunc)):
                    np.testing.assert_array_equal(np_(got), exp[name], where + " " + name)
                fg = orc.split_obs(np_(obs._packed), A, O)
                fo = orc.split_obs(exp["obs"], A, O)
                assert_obs_close(fg, dict(zip(OBS_FIELDS, fo)), prefix="", exact=True, where=where)
                st, ob, tg, sn, te = (exp[x] for x in ("states", "obstacles", "target",
                                                       "step_num", "terminates"))
            ran.add(got_fam)
            o2 = env.observations()  # observe-only instantiation of the same family
            torch.cuda.synchronize()
            assert lib.marlnav_debug_last_family() == got_fam
            fg = orc.split_obs(np_(o2._packed), A, O)
            assert_obs_close(fg, dict(zip(OBS_FIELDS, orc.split_obs(exp["obs"], A, O))),
                             prefix="", exact=True, where=where + " observe")
        finally:
            lib.marlnav_debug_force_family(prev)
    assert ran == expect, (sorted(ran), sorted(expect))


@pytest.mark.parametrize("shape", [(20000 + 3, 3, 3), (512, 16, 32)])
@pytest.mark.parametrize("geom", [
    dict(_init_dist=7.0, _bond_sharpness=0.05, _ideal_dist=33.3, _max_at_prop_d=3),  # fast terms
    dict(_init_dist=3.0e7, _bond_sharpness=0.01, _ideal_dist=1e-30),                   # IEEE terms
    dict(_bond_sharpness=1e6, _ideal_dist=0.0, _max_at_prop_d=1.5e-6),                 # boundaries
    dict(_bond_sharpness=0.25, _max_at_prop_d=-4.0, _ideal_dist=-12.0),                # powers of 2
])
def test_reward_term_divisions_bit_exact_for_any_parameters(pkg, geom, shape):
    """The reward terms divide by parameters (environment.py:236-269); the
    kernels use the short exact division sequences only when the host finds
    every such parameter inside their guards (marlnav_step, terms_fast_params)
    and IEEE division otherwise (the block kernel; the split kernel, the
    second shape, for its bond terms). Rewards stay bit-exact vs the oracle
    (which divides with IEEE division) either way."""
    P, A, O = shape
    g = torch.Generator().manual_seed(77)
    env = make_env(pkg, P, A, O, episode_len=40, seed=3,
                   factors=dict(risk_factor=1.5, distance_factor=3., soft_factor=7.,
                                bond_factor=11.))
    for k, v in geom.items():
        setattr(env, k, v)
    dm, pr = oracle_params(env)
    form = np_(env._formation)
    st, ob, tg = (np_(x).copy() for x in (env.states, env.obstacles, env.target))
    sn = np.zeros(P, np.float32)
    te = np.zeros(P, np.bool_)
    for k in range(4):
        acts = ((torch.rand(P, A, 2, generator=g) - 0.5) * 0.8).numpy()
        exp = orc.step(dm, pr, st, ob, tg, sn, te, acts, formation=form, step_idx=k + 1)
        obs, rew, term, trunc = env.step(torch.from_numpy(acts).to(DEV))
        where = f"{geom} step {k + 1}"
        np.testing.assert_array_equal(np_(rew), exp["reward"], where)
        np.testing.assert_array_equal(np_(env.states), exp["states"], where)
        st, ob, tg, sn, te = (exp[x] for x in ("states", "obstacles", "target", "step_num",
                                               "terminates"))


@pytest.mark.parametrize("P,A,O", [(4096 + 7, 3, 3), (300, 3, 3), (60, 3, 3), (512, 16, 32)])
def test_non_finite_inputs_match_oracle(pkg, P, A, O):
    """NaN / inf actions and state entries propagate exactly as in the oracle
    (torch.clamp passes NaN, comparisons with NaN are false): states, rewards
    and flags equal bit for bit, NaN for NaN (block, split and LPR=8 split
    kernels; the non-finite blocks take the IEEE pair math)."""
    g = torch.Generator().manual_seed(P + 5)
    env = make_env(pkg, P, A, O, episode_len=50, seed=9)
    st = env.states.cpu().clone()
    st[3, 0, 0] = float("nan")
    st[9, 1, 2:4] = torch.tensor([float("inf"), 0.0])
    st[17, 2, 4] = float("-inf")
    env.states = st
    dm, pr = oracle_params(env)
    form = np_(env._formation)
    s, o, t = st.numpy(), np_(env.obstacles).copy(), np_(env.target).copy()
    sn = np.zeros(P, np.float32)
    te = np.zeros(P, np.bool_)
    for k in range(3):
        acts = ((torch.rand(P, A, 2, generator=g) - 0.5) * 0.8)
        acts[5, 0, 0] = float("nan")
        acts[40, 1, 1] = float("inf")
        acts[41, 0, 0] = float("-inf")
        acts = acts.numpy()
        exp = orc.step(dm, pr, s, o, t, sn, te, acts, formation=form, step_idx=k + 1)
        obs, rew, term, trunc = env.step(torch.from_numpy(acts).to(DEV))
        where = f"P{P} A{A} O{O} step {k + 1}"
        for name, got in (("states", env.states), ("obstacles", env.obstacles),
                          ("step_num", env._step_num), ("terminates", env._terminates),
                          ("reward", rew), ("terminated", term), ("truncated", trunc)):
            np.testing.assert_array_equal(np_(got), exp[name], where + " " + name)
        got = np_(obs._packed)
        assert np.array_equal(np.isnan(got), np.isnan(exp["obs"])), where + " NaN pattern"
        fg, fo_ = orc.split_obs(got, A, O), orc.split_obs(exp["obs"], A, O)
        assert_obs_close(fg, dict(zip(OBS_FIELDS, fo_)), prefix="", exact=True, where=where)
        s, o, t, sn, te = (exp[x] for x in ("states", "obstacles", "target", "step_num",
                                            "terminates"))


@pytest.mark.parametrize("P,A,O", [(2 * 1048576 + 37, 3, 3), (131072, 3, 8), (4096, 16, 32)])
def test_full_size_slices_bit_exact_vs_oracle(pkg, P, A, O):
    """Beyond BASELINE sizes (2^21 envs per GPU, ragged): envs are
    independent and the native re-init is keyed by the global env id, so the
    oracle stepping a contiguous slice (env_offset = its first env) must
    reproduce the kernel's results on that slice exactly. Slices at the
    start, in the middle and at the ragged end; 2-step episodes so most envs
    re-initialise."""
    g = torch.Generator(device=DEV).manual_seed(P)
    env = make_env(pkg, P, A, O, episode_len=2, seed=31)
    env._sync_params()
    pr = env._cparams
    form = np_(env._formation)
    n = min(4096, P // 4)
    starts = [0, P // 2 - n // 4, P - n]
    cur = [tuple(np_(x[s:s + n]).copy() for x in (env.states, env.obstacles, env.target))
           + (np.zeros(n, np.float32), np.zeros(n, np.bool_)) for s in starts]
    for k in range(3):
        acts = (torch.rand(P, A, 2, generator=g, device=DEV) - 0.5) * 0.8
        obs, rew, term, trunc = env.step(acts)
        for i, s in enumerate(starts):
            dm = orc.make_dims(n, A, O, env_offset=s)
            st, ob, tg, sn, te = cur[i]
            exp = orc.step(dm, pr, st, ob, tg, sn, te, np_(acts[s:s + n]), formation=form,
                           step_idx=k + 1)
            where = f"P{P} slice {s} step {k + 1}"
            for name, got in (("states", env.states), ("obstacles", env.obstacles),
                              ("target", env.target), ("step_num", env._step_num),
                              ("terminates", env._terminates), ("reward", rew),
                              ("terminated", term), ("truncated", trunc)):
                np.testing.assert_array_equal(np_(got[s:s + n]), exp[name], where + " " + name)
            fg = orc.split_obs(np_(obs._packed[s:s + n]), A, O)
            assert_obs_close(fg, dict(zip(OBS_FIELDS, orc.split_obs(exp["obs"], A, O))),
                             prefix="", exact=True, where=where)
            cur[i] = tuple(exp[x] for x in ("states", "obstacles", "target", "step_num",
                                            "terminates"))


def _run_vs_oracle(env, dm, pr, st, ob, tg, sn, te, acts_list, form=None, fresh_list=None,
                   where=""):
    """Step env and the oracle side by side; every output bit for bit
    (NaN for NaN). Returns the final state."""
    for k, acts in enumerate(acts_list):
        fresh = fresh_list[k] if fresh_list is not None else None
        if fresh is not None:
            env._init_sampler = lambda fr=fresh: tuple(torch.from_numpy(x) for x in fr)
        exp = orc.step(dm, pr, st, ob, tg, sn, te, acts, formation=form, fresh=fresh,
                       step_idx=k + 1)
        obs, rew, term, trunc = env.step(torch.from_numpy(acts).to(DEV))
        w = f"{where} step {k + 1}"
        for name, got in (("states", env.states), ("obstacles", env.obstacles),
                          ("target", env.target), ("step_num", env._step_num),
                          ("terminates", env._terminates), ("reward", rew),
                          ("terminated", term), ("truncated", trunc)):
            np.testing.assert_array_equal(np_(got), exp[name], w + " " + name)
        A, O = dm.num_agents, dm.num_obstacles
        fg, fo = orc.split_obs(np_(obs._packed), A, O), orc.split_obs(exp["obs"], A, O)
        assert_obs_close(fg, dict(zip(OBS_FIELDS, fo)), prefix="", exact=True, where=w)
        st, ob, tg, sn, te = (exp[x] for x in ("states", "obstacles", "target", "step_num",
                                                "terminates"))
    return st, ob, tg, sn, te


@pytest.mark.parametrize("P,A,O", [(4096 + 7, 3, 3), (300, 3, 3), (60, 3, 3), (2048, 3, 8), (512, 16, 32),
                                   (777, 5, 2)])
def test_non_finite_env_reinitialised_like_the_reference_blend(pkg, P, A, O):
    """_reinit_update (environment.py:86-90) is 0*old + 1*fresh for a
    finished env: an env whose state, obstacle or target holds NaN/inf stays
    NaN where it did after its re-init, in every kernel family's native
    re-init path. 2-step episodes: every env re-initialises at step 2; the
    oracle restates the reference's blend (pinned to the reference's own
    expression in tests/test_oracle_golden.py)."""
    g = torch.Generator().manual_seed(P + 3)
    env = make_env(pkg, P, A, O, episode_len=2, seed=13)
    st = env.states.cpu().clone()
    ob = env.obstacles.cpu().clone()
    tg = env.target.cpu().clone()
    st[3, 0, 0] = float("nan")
    st[9, 1, 2:4] = torch.tensor([float("inf"), 0.0])
    st[17, A - 1, 4] = float("-inf")
    ob[40, 0, 1] = float("nan")
    tg[55, 0, 0] = float("inf")
    st[P - 1, 0, 3] = float("nan")
    env.states, env.obstacles, env.target = st, ob, tg
    dm, pr = oracle_params(env)
    form = np_(env._formation)
    acts = [((torch.rand(P, A, 2, generator=g) - 0.5) * 0.8).numpy() for _ in range(4)]
    _run_vs_oracle(env, dm, pr, st.numpy(), ob.numpy(), tg.numpy(), np.zeros(P, np.float32),
                   np.zeros(P, np.bool_), acts, form=form, where=f"P{P} A{A} O{O}")


@pytest.mark.parametrize("P,A,O", [(20000 + 13, 3, 3), (300, 3, 3), (60, 3, 3), (512, 16, 32)])
def test_reference_rng_non_finite_fresh_candidates(pkg, P, A, O):
    """Reference-RNG mode with a sampler that returns NaN/inf candidates:
    the reference's blend makes a KEPT env's value NaN too (1*old +
    0*inf); a finished env takes the candidate (0*old + inf). Host fix-up
    of the kept envs + re-observation, vs the oracle."""
    g = torch.Generator().manual_seed(P * 3 + O)
    env = make_env(pkg, P, A, O, episode_len=3, rng="reference", noise_device="cpu")
    dm, pr = oracle_params(env)
    st, ob, tg = (np_(x).copy() for x in (env.states, env.obstacles, env.target))
    fresh_list, acts = [], []
    for k in range(4):
        fs = (torch.rand(P, A, 5, generator=g) * 900.0).numpy()
        fo = (torch.rand(P, O, 2, generator=g) * 700.0).numpy()
        ft = (torch.rand(P, 1, 2, generator=g) * 1400.0).numpy()
        if k in (1, 2):
            fs[5 + k, 0, 1] = float("nan")
            fo[11, O - 1, 0] = float("inf")
            ft[P - 2, 0, 1] = float("-inf")
        fresh_list.append((fs, fo, ft))
        acts.append(((torch.rand(P, A, 2, generator=g) - 0.5) * 0.9).numpy())
    _run_vs_oracle(env, dm, pr, st, ob, tg, np.zeros(P, np.float32), np.zeros(P, np.bool_),
                   acts, fresh_list=fresh_list, where=f"P{P} A{A} O{O}")


@pytest.mark.parametrize("shape", [(5000 + 3, 3, 3, 9), (600, 16, 32, 2)])
@pytest.mark.parametrize("cap", [50.0, 0.0, 1e6])
def test_cap_distance_reaches_step_and_observe(pkg, cap, shape):
    """env._cap_distance (environment.py:65) caps the angles in step AND in
    observations()/reset() (environment.py:172-177), like the reference;
    with 2-step episodes also in the re-observation of re-initialised envs
    (at A16/O32 through the formation template, whose bearings are stored
    uncapped)."""
    P, A, O, ep = shape
    g = torch.Generator().manual_seed(7)
    env = make_env(pkg, P, A, O, episode_len=ep, seed=4)
    env._cap_distance = cap
    dm, pr = oracle_params(env)
    assert abs(pr.cap_distance - cap) <= 1e-6 * max(cap, 1.0)
    form = np_(env._formation)
    st, ob, tg = (np_(x).copy() for x in (env.states, env.obstacles, env.target))
    exp0 = orc.observe(dm, st, ob, tg, params=pr)
    fg = orc.split_obs(np_(env.observations()._packed), A, O)
    assert_obs_close(fg, dict(zip(OBS_FIELDS, orc.split_obs(exp0, A, O))), prefix="",
                     exact=True, where="observe")
    acts = [((torch.rand(P, A, 2, generator=g) - 0.5) * 0.8).numpy() for _ in range(3)]
    _run_vs_oracle(env, dm, pr, st, ob, tg, np.zeros(P, np.float32), np.zeros(P, np.bool_),
                   acts, form=form, where=f"cap {cap}")
    if cap >= 1e6:  # every angle capped
        assert float(env.observations().target_angle.abs().max()) == 0.0


def test_fused_action_scaler_vs_oracle(pkg):
    """§8(f) row 2 against the oracle: raw policy actions in [-1, 1] through
    the ActionScaler fused into the kernel's action load (utils.py:535-547)
    equal the oracle stepping with the same scale/mean (MARLNAV_SCALE_ACTIONS)."""
    P, A, O = 3000 + 1, 3, 3
    args = cli_args(num_parallel=P, num_obstacles=O)
    scl = pkg.ActionScaler(pkg.set_scaler_params(args, DEV))
    env = make_env(pkg, P, A, O, episode_len=12, seed=8)
    env.attach_action_scaler(scl)
    dm, pr = oracle_params(env)
    assert pr.flags & pkg.abi.SCALE_ACTIONS
    np.testing.assert_array_equal(np.array(pr.act_scale, np.float32),
                                  np_(scl.scale).astype(np.float32).reshape(-1))
    form = np_(env._formation)
    g = torch.Generator().manual_seed(12)
    st, ob, tg = (np_(x).copy() for x in (env.states, env.obstacles, env.target))
    acts = [(torch.rand(P, A, 2, generator=g) * 2 - 1).numpy() for _ in range(20)]
    _run_vs_oracle(env, dm, pr, st, ob, tg, np.zeros(P, np.float32), np.zeros(P, np.bool_),
                   acts, form=form, where="scaled")


def test_configs4_sharded_slices_equal_one_batch_and_oracle(pkg):
    """BASELINE configs[4]: 131072 envs x 3 agents x 3 obstacles as eight
    independent 16384-env slices (env_offset = r * 16384, one per GPU in the
    8-GPU run; all on this GPU here), 20 steps: every slice equals the
    matching rows of one 131072-env Env bit for bit (native re-init keyed by
    the global env id), and the oracle on each slice's first and last 64
    envs."""
    n, R, A, O = 16384, 8, 3, 3
    P = n * R
    full = make_env(pkg, P, A, O, episode_len=7, seed=2026,
                    factors=dict(risk_factor=2., distance_factor=3.))
    shards = [make_env(pkg, n, A, O, episode_len=7, seed=2026, env_offset=r * n,
                       factors=dict(risk_factor=2., distance_factor=3.)) for r in range(R)]
    for r, e in enumerate(shards):
        assert torch.equal(e.states, full.states[r * n:(r + 1) * n])
        assert torch.equal(e.obstacles, full.obstacles[r * n:(r + 1) * n])
    full._sync_params()
    pr = full._cparams
    form = np_(full._formation)
    cur = {}
    for r in range(R):
        for s0 in (r * n, (r + 1) * n - 64):
            cur[s0] = tuple(np_(x[s0:s0 + 64]).copy() for x in (full.states, full.obstacles,
                                                                full.target)) + (
                np.zeros(64, np.float32), np.zeros(64, np.bool_))
    g = torch.Generator(device=DEV).manual_seed(44)
    for k in range(20):
        acts = (torch.rand(P, A, 2, generator=g, device=DEV) - 0.5) * 0.8
        fo, fr, fte, ftr = full.step(acts)
        for r, e in enumerate(shards):
            so, sr, ste, stt = e.step(acts[r * n:(r + 1) * n])
            sl = slice(r * n, (r + 1) * n)
            where = f"shard {r} step {k + 1}"
            assert torch.equal(e.states, full.states[sl]), where
            assert torch.equal(e.obstacles, full.obstacles[sl]), where
            assert torch.equal(sr, fr[sl]) and torch.equal(ste, fte[sl]), where
            assert torch.equal(stt, ftr[sl]), where
            assert torch.equal(so._packed, fo._packed[sl]), where
        for s0, (st, ob, tg, sn, te) in list(cur.items()):
            dm = orc.make_dims(64, A, O, env_offset=s0)
            exp = orc.step(dm, pr, st, ob, tg, sn, te, np_(acts[s0:s0 + 64]), formation=form,
                           step_idx=k + 1)
            where = f"oracle slice {s0} step {k + 1}"
            for name, got in (("states", full.states), ("obstacles", full.obstacles),
                              ("reward", fr), ("terminated", fte), ("truncated", ftr)):
                np.testing.assert_array_equal(np_(got[s0:s0 + 64]), exp[name], where + name)
            fg = orc.split_obs(np_(fo._packed[s0:s0 + 64]), A, O)
            assert_obs_close(fg, dict(zip(OBS_FIELDS, orc.split_obs(exp["obs"], A, O))),
                             prefix="", exact=True, where=where)
            cur[s0] = tuple(exp[x] for x in ("states", "obstacles", "target", "step_num",
                                             "terminates"))
    tot = np.sum([[e._num_trunc, e._num_col, e._num_tar] for e in shards], axis=0)
    assert tot.tolist() == [full._num_trunc, full._num_col, full._num_tar]
    assert tot[0] > 0 and tot[1] > 0


def test_mappo_get_data_rollout_matches_reference(pkg):
    """F6: the reference's MAPPO.get_data loop (models.py:106-129: normalise
    observations, step with up-scaled policy actions, keep obs / actions /
    log-probs / values / rewards / done, then _process_rewards) run on the
    drop-in Env with the fused ObsNormalizer and ActionScaler and the device
    RolloutBuffer, reference-RNG mode: 200 steps of normalised observations,
    rewards and done flags and the processed returns against the reference's
    (trajectory tolerances: tests/conftest.py assert_traj_obs_close)."""
    import math
    from conftest import assert_traj_obs_close
    m, z = meta("rollout_getdata"), golden("rollout_getdata")
    P, A, O, T = m["num_parallel"], 3, 3, m["buffer_len"]
    args = cli_args(num_parallel=P, episode_len=m["episode_len"], risk_factor=m["risk_factor"],
                    distance_factor=m["distance_factor"], buffer_len=T, gamma=m["gamma"])
    nrm = pkg.ObsNormalizer(pkg.set_normalizer_params(args, DEV))
    scl = pkg.ActionScaler(pkg.set_scaler_params(args, DEV))
    pkg.set_all_seeds(m["seed"])
    params = pkg.set_env_params(args, DEV)
    params["init"] = dict(params["init"], noise_device="cpu")
    params["rng"] = "reference"
    env = pkg.Env(params)
    np.testing.assert_array_equal(np_(env.states), z["states0"])
    env.attach_normalizer(nrm)
    env.attach_action_scaler(scl)
    pkg.set_all_seeds(m["reseed"])
    obs_n = nrm(env.observations())
    buf = pkg.rollout.RolloutBuffer(T)
    for t in range(T):
        assert_traj_obs_close(np_(obs_n), z["obs_norm"][t], A, O, angle_scale=math.pi,
                              what=f"obs_norm {t}")
        raw = torch.from_numpy(z["actions"][t]).to(DEV)
        obs, rew, term, trunc = env.step(raw.view(P, A, 2))       # scaled in the kernel
        done = torch.logical_or(term, trunc)
        np.testing.assert_array_equal(np_(done), z["done"][t], f"done {t}")
        assert_vec_close(np_(rew), z["reward"][t], atol=1e-4, what=f"reward {t}")
        buf.add(obs_n, raw, torch.zeros(P * A, device=DEV), torch.zeros(P, 1, device=DEV),
                rew, done)
        obs_n = nrm(obs)
        assert obs_n is obs._normalized                             # the fused copy
    assert_traj_obs_close(np_(obs_n), z["final_obs_norm"], A, O, angle_scale=math.pi,
                          what="final obs")
    mean = buf.process_rewards(m["gamma"])
    ret = np.stack([np_(e[4]) for e in buf.entries()])
    np.testing.assert_allclose(ret, z["returns"], rtol=1e-5, atol=1e-6)
    assert abs(float(mean) - float(z["mean_rew"])) <= 1e-5 * abs(float(z["mean_rew"]))
    assert (env._num_trunc, env._num_col, env._num_tar) == (m["num_trunc"], m["num_col"],
                                                            m["num_tar"])


def test_graph_capture_needs_explicit_opt_in(pkg):
    """A captured Env.step bakes its re-init draws into the graph:
    capture raises unless env.allow_graph_capture is set; with it, replays
    run the captured step (bench.py's kernel_time_us)."""
    env = make_env(pkg, 1024, 3, 3, episode_len=200, seed=3)
    acts = torch.zeros(1024, 3, 2, device=DEV)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        env.step(acts)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    assert not env.allow_graph_capture
    g = torch.cuda.CUDAGraph()
    with warnings.catch_warnings():  # torch notes the aborted capture is empty
        warnings.simplefilter("ignore", UserWarning)
        with pytest.raises(RuntimeError, match="allow_graph_capture"):
            with torch.cuda.graph(g):
                env.step(acts)
    torch.cuda.synchronize()
    env.allow_graph_capture = True
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = env.step(acts)
    before = np_(env.states).copy()
    g.replay()
    torch.cuda.synchronize()
    assert not np.array_equal(np_(env.states), before)   # the replay stepped the env
    assert out[1].shape == (1024,)


@pytest.mark.parametrize("P,A,O", [(4096, 3, 3), (4096 + 37, 3, 3), (2048 + 5, 3, 8)])
def test_collisions_at_the_threshold_ulp_bit_exact_vs_oracle(pkg, P, A, O):
    """Collision tests d < c (environment.py:207-214) on distances from the
    env-block kernel's short correctly rounded sqrt, at the threshold's ulp:
    agent-obstacle distances within +-8 ulps of ob_coll_dist and agent-agent
    distances within +-8 ulps of ag_coll_dist, one offset per env (full and
    ragged last blocks, O3 and O8): terminated flags, re-initialised states
    and the re-observed rows equal the oracle's bit for bit."""
    env = make_env(pkg, P, A, O, episode_len=50, seed=21)
    e = np.arange(P)
    k = (e % 17) - 8                         # ulp offset of this env
    st = np.zeros((P, A, 5), np.float32)
    st[:, :, 0] = -3.0                        # heading +x, speed 3, turn 0, accel 0:
    st[:, :, 2] = 1.0                         # every agent moves exactly to x = 0
    st[:, :, 4] = 3.0
    st[:, 0, 1] = 0.0
    st[:, 1, 1] = 1000.0
    st[:, 2, 1] = 2000.0
    pair = e % 3 == 1                         # every third env: agents 0, 1 at ~5
    y1 = np.float32(5.0) + k.astype(np.float32) * np.float32(2.0 ** -21)
    st[pair, 1, 1] = y1[pair]
    ob = np.full((P, O, 2), 4000.0, np.float32)
    ob[:, :, 1] += np.arange(O, dtype=np.float32) * 100.0
    near = e % 3 != 1                         # the others: obstacle 0 at ~50 from agent 0
    ob[near, 0, 0] = (np.float32(50.0) + k.astype(np.float32) * np.float32(2.0 ** -18))[near]
    ob[near, 0, 1] = 0.0
    tg = np.full((P, 1, 2), -5000.0, np.float32)
    env.states = torch.from_numpy(st)
    env.obstacles = torch.from_numpy(ob)
    env.target = torch.from_numpy(tg)
    dm, pr = oracle_params(env)
    form = np_(env._formation)
    acts = [np.zeros((P, A, 2), np.float32) for _ in range(2)]
    sn = np.zeros(P, np.float32)
    te = np.zeros(P, np.bool_)
    exp1 = orc.step(dm, pr, st, ob, tg, sn, te, acts[0], formation=form, step_idx=1)
    n_col = int(exp1["terminated"].sum())
    assert 0.3 * P < n_col < 0.7 * P, n_col   # both sides of the threshold are hit
    lib = env._lib
    prev = lib.marlnav_debug_force_family(1)  # MARLNAV_FAMILY_BLOCK
    try:
        _run_vs_oracle(env, dm, pr, st, ob, tg, sn, te, acts, form=form,
                       where=f"P{P} A{A} O{O}")
        assert lib.marlnav_debug_last_family() == 1
    finally:
        lib.marlnav_debug_force_family(prev)


@pytest.mark.parametrize("P,A,O,steps", [(20000 + 3, 3, 3, 12), (512, 16, 32, 6)])
def test_c_host_matches_python_env(pkg, P, A, O, steps, tmp_path):
    """The C ABI without Python or torch: examples/c_host/step_loop (C++, HIP
    runtime + libmarlnav.so) initialises the envs (marlnav_reinit_all), steps
    them with the given actions (marlnav_step per step, the native re-init
    keyed by the step index) and sums the counters; the Python Env with the
    same dims, parameters, seed and actions ends bit for bit in the same
    state, last outputs and counters (5-step episodes: re-inits happen)."""
    exe = os.path.join(ROOT, "examples", "c_host", "step_loop")
    assert os.path.exists(exe), "examples/c_host/step_loop not built (__graft_entry__.build)"
    env = make_env(pkg, P, A, O, episode_len=5, seed=2024,
                   factors=dict(risk_factor=2., distance_factor=3., bond_factor=5.))
    env._sync_params()
    acts = ((np.random.default_rng(P + A).random((steps, P, A, 2), dtype=np.float32) - 0.5)
            * np.float32(0.8)).astype(np.float32)
    inp, out = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(inp, "wb") as f:
        f.write(bytes(env._dims))
        f.write(bytes(env._cparams))
        f.write(np.int32(steps).tobytes())
        f.write(np_(env._formation).astype(np.float32).tobytes())
        f.write(acts.tobytes())
    r = subprocess.run([exe, str(inp), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    for k in range(steps):
        obs, rew, term, trunc = env.step(torch.from_numpy(acts[k]).to(DEV))
    torch.cuda.synchronize()
    D = 2 + 2 * O + 2 * (A - 1)
    raw = out.read_bytes()
    parts = [("states", np.float32, (P, A, 5), env.states), ("obstacles", np.float32, (P, O, 2), env.obstacles),
             ("target", np.float32, (P, 1, 2), env.target), ("step_num", np.float32, (P,), env._step_num),
             ("terminates", np.uint8, (P,), env._terminates), ("obs", np.float32, (P, A, D), obs._packed),
             ("reward", np.float32, (P,), rew), ("terminated", np.uint8, (P,), term),
             ("truncated", np.uint8, (P,), trunc)]
    off = 0
    for name, dt, shape, got in parts:
        n = int(np.prod(shape)) * np.dtype(dt).itemsize
        c = np.frombuffer(raw[off:off + n], dtype=dt).reshape(shape)
        off += n
        g = np_(got)
        g = g.astype(np.uint8) if dt == np.uint8 else g
        assert g.shape == c.shape, (name, g.shape, c.shape)
        np.testing.assert_array_equal(g.view(np.uint32) if dt == np.float32 else g,
                                      c.view(np.uint32) if dt == np.float32 else c, name)
    counters = np.frombuffer(raw[off:off + 24], dtype=np.uint64)
    assert off + 24 == len(raw)
    assert tuple(int(x) for x in counters) == (env._num_trunc, env._num_col, env._num_tar)
    assert counters[0] > 0  # the 5-step episodes truncated


@pytest.mark.parametrize("P,A,O", [(4096, 3, 3), (2048 + 5, 3, 8), (60, 3, 3), (512, 16, 32),
                                   (16384, 3, 3), (16001, 3, 3)])
def test_fused_normalizer_every_store_path(pkg, P, A, O):
    """The fused normaliser (MARLNAV_WRITE_OBS_NORM, utils.py:519-532) in
    every store path: the env-block kernel's per-thread-feature path (A3/O3
    full blocks), its generic path (A3/O8: D does not divide the block), the
    draw-wave instantiation (at most one block per CU: 16384 full blocks, and
    16001 whose ragged last block takes the generic path, whose barrier the
    draw wave must meet), the pair-split kernel (LPR 8 at 60 envs, A16/O32):
    the fused output equals
    (obs - mean) / scale in torch bit for bit, with a mean and scale per
    feature (re-inits included: 4-step episodes)."""
    from types import SimpleNamespace
    D = 2 + 2 * O + 2 * (A - 1)
    g = torch.Generator().manual_seed(P + D)
    mean = (torch.rand(D, generator=g) * 100 - 50).to(DEV)
    scale = (torch.rand(D, generator=g) * 900 + 0.5).to(DEV)
    env = make_env(pkg, P, A, O, episode_len=4, seed=7)
    env.attach_normalizer(SimpleNamespace(mean=mean, scale=scale))
    for k in range(6):
        acts = ((torch.rand(P, A, 2, generator=g) - 0.5) * 0.8).to(DEV)
        obs, rew, term, trunc = env.step(acts)
        ref = (obs._packed - mean) / scale
        torch.testing.assert_close(obs._normalized, ref, rtol=0, atol=0,
                                   msg=f"P{P} A{A} O{O} step {k + 1}")


@pytest.mark.parametrize("first,n", [
    (0x00000000, 1 << 20),            # +0 and the smallest magnitudes
    (0x3EFF0000, 1 << 18),            # around |x| = 0.5 (the branch point)
    (0x3F7C0000, (1 << 18) + 1),      # the last 2^18 floats below 1, and 1
    (0x80000000, 1 << 16),            # -0 and tiny negatives
    (0xBF7E0000, (1 << 17) + 1),      # down to -1
])
def test_kernel_acos_equals_oracle_restatement(pkg, first, n):
    """The step kernels' bearing acos (acos_k through marlnav_debug_acos_range)
    equals the oracle's acos_device bit for bit on contiguous runs of fp32
    inputs (environment.py:286). tests/golden/acos_dev_check.py sweeps all
    2 130 706 434 inputs in [-1, 1] (profiles/r04_acos_device.json)."""
    lib = pkg.abi.load_library()
    out = torch.empty(n, dtype=torch.float32, device=DEV)
    assert lib.marlnav_debug_acos_range(first, n, out.data_ptr(), None) == 0
    got = np_(out)
    exp = orc.acos_device_range(first, n)
    bad = np.flatnonzero(got.view(np.uint32) != exp.view(np.uint32))
    assert bad.size == 0, (f"{bad.size} of {n} differ, first at bits "
                           f"{first + int(bad[0]):#010x}: {got[bad[0]]!r} vs {exp[bad[0]]!r}")


@pytest.mark.parametrize("d_first,d_stride,nd", [
    (0, 127, 65536),             # 1/128 of the divisor significands, spread over [1, 2)
    (0x7FFFFF - 255, 1, 256),    # the last 256, up to the all-ones significand
    (0, 1, 256),                 # 1.0 and its neighbours
])
def test_fast_division_sequences_exact(pkg, d_first, d_stride, nd):
    """The kernels' short division sequences (div2_fast / div_c: one Newton
    step and ONE residual correction; recip_fast: the Newton step alone)
    against IEEE division, through marlnav_debug_fastdiv_check, for every
    dividend significand of each sampled divisor: zero mismatches. Inside the
    guards the sequences are scale- and sign-invariant, so significand pairs
    decide every case; scripts/probes/div_exhaustive.hip checks all 2^46
    (profiles/r05_div_exhaustive.txt)."""
    lib = pkg.abi.load_library()
    out = torch.zeros(3, dtype=torch.int64, device=DEV)  # (65536 x 2^23 pairs: ~0.3 s)
    assert lib.marlnav_debug_fastdiv_check(d_first, d_stride, nd, out.data_ptr(), None) == 0
    got = [int(v) for v in np_(out)]
    assert got == [0, 0, 0], (f"mismatches over {nd} divisors x 2^23 dividends: quotients {got[0]}, "
                              f"parameter divisions {got[1]}, reciprocals {got[2] & 0xFFFFFFFF}, "
                              f"guard refusals {got[2] >> 32}")


def test_kernel_acos_strided_sample(pkg):
    """Every 997th fp32 of [-1, 1] through the kernels' acos vs the oracle's,
    evaluated in chunks of 2^24 consecutive patterns (64 MB of device output
    at a time; only the sampled entries are kept)."""
    lib = pkg.abi.load_library()
    step, ch = 997, 1 << 24
    out = torch.empty(ch, dtype=torch.float32, device=DEV)
    for base in (0, 0x80000000):
        bits = np.arange(base, base + 0x3F800001, step, dtype=np.uint64).astype(np.uint32)
        exp = orc.acos_device(bits.view(np.float32))
        total = int(bits[-1] - bits[0]) + 1
        parts = []
        for off in range(0, total, ch):
            n = min(ch, total - off)
            assert lib.marlnav_debug_acos_range(int(bits[0]) + off, n, out.data_ptr(), None) == 0
            parts.append(np_(out[(-off) % step:n:step]))
        got = np.concatenate(parts)
        assert got.size == exp.size
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))