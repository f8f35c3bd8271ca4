"""Distributional parity of the native re-init (rng='native', the default
and the bench's mode) with the reference's sampler, TriangleIntitializer
(marlnav/utils.py:381-398): fresh obstacles and noisy agents from the oracle
(CPU) and from the GPU kernels (the initial-state kernel and the in-step
re-init of every kernel family) against the reference's law. See
tests/rng_stats.py for what is checked and why."""
import json

import numpy as np
import pytest
import torch

from conftest import cli_args, env_values, meta

import oracle as orc
import rng_stats as rs

SEED = 20251003


def reference_sample(pkg, P, O, noisy=False, seed=7):
    """Draws of the reference's own sampler law: the host TriangleIntitializer
    in reference-RNG mode (torch.rand / normal_ on the CPU, pinned draw for
    draw to the reference by F4)."""
    pkg.set_all_seeds(seed)
    p = dict(pkg.set_init_params(cli_args(num_parallel=P, num_obstacles=O), "cpu"))
    p["noisy_ags"] = noisy
    smp = pkg.init_sampler(p)
    st, ob, _ = smp()
    return smp, st.numpy(), ob.numpy()


def init_consts(smp):
    return (smp._obs_x_range, smp._obs_mean_x, smp._obs_y_range, smp._obs_mean_y)


def _print(tag, d):
    print(tag, json.dumps(d, sort_keys=True))


# ------------------------------------------------------------------ CPU twin
@pytest.mark.parametrize("P,O", [(1 << 18, 3), (1 << 15, 32)])
def test_oracle_native_obstacles_follow_reference_law(pkg, P, O):
    """The oracle's native stream (the restatement the GPU kernels are
    checked against bit for bit): >= 1.5e6 coordinates on the reference's
    24-bit grid image, uniform, uncorrelated, and the same law as the
    reference sampler's draws (two-sample KS), at the initial state (step 0)
    and at a later step's re-init draws."""
    import marlnav_amd.environment as envmod
    smp, _, ref_ob = reference_sample(pkg, 1 << 16, O)
    form = np.concatenate([smp.formation.reshape(-1).numpy(),
                           smp.target_point.reshape(-1).numpy()]).astype(np.float32)
    pr = envmod.make_cparams(env_values(meta("step_a3o3")), init=smp, seed=SEED)
    dm = orc.make_dims(P, 3, O)
    _, ob0, _ = orc.reinit_all(dm, pr, form, 0)
    _, ob9, _ = orc.reinit_all(dm, pr, form, 9)
    c = init_consts(smp)
    _print(f"oracle native P{P} O{O} step 0", rs.check_obstacles(ob0, *c, ref=ref_ob))
    _print(f"oracle native P{P} O{O} step 9", rs.check_obstacles(ob9, *c, ref=ref_ob))
    rs.check_uncorrelated(ob0[..., 0], ob9[..., 0], "step 0 vs step 9")
    assert np.count_nonzero(ob0 == ob9) < 1e-4 * ob0.size


def test_oracle_native_noisy_agents_follow_reference_law(pkg):
    """Noisy agents (utils.py:381-388) from the oracle's native stream:
    Gaussian position noise and uniform heading angles of the reference's
    scale, and the same law as the reference sampler's noise (KS)."""
    import marlnav_amd.environment as envmod
    P = 1 << 17
    smp, ref_st, _ = reference_sample(pkg, 1 << 16, 3, noisy=True)
    form = np.concatenate([smp.formation.reshape(-1).numpy(),
                           smp.target_point.reshape(-1).numpy()]).astype(np.float32)
    pr = envmod.make_cparams(env_values(meta("step_a3o3")), init=smp, seed=SEED)
    st, _, _ = orc.reinit_all(orc.make_dims(P, 3, 3), pr, form, 0)
    _print("oracle native noisy agents", rs.check_noisy_agents(
        st, smp.formation.numpy(), smp.ags_dist, smp.ags_std, smp.angle_range, ref=ref_st))
    # and the reference's own draws pass the same checks (the checker is sound)
    rs.check_noisy_agents(ref_st, smp.formation.numpy(), smp.ags_dist, smp.ags_std,
                          smp.angle_range)


def test_reference_sampler_passes_the_same_checks(pkg):
    """The checks themselves, on the reference sampler's own draws: on the
    grid image, uniform and uncorrelated (a checker that rejected the
    reference would prove nothing)."""
    smp, _, ref_ob = reference_sample(pkg, 1 << 18, 3, seed=11)
    _print("reference sampler", rs.check_obstacles(ref_ob, *init_consts(smp)))


# ----------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("P,A,O", [(1 << 19, 3, 3), (1 << 16, 3, 8), (4096, 16, 32)])
def test_gpu_native_draws_follow_reference_law(pkg, P, A, O):
    """Fresh obstacles as the GPU draws them: the initial-state kernel
    (marlnav_reinit_all) and the in-step re-init of finished envs (block
    kernel stage-time draws at A3/O3, the per-env pass at A3/O8, the split
    kernel's one-pass re-init at A16/O32). episode_len 1 makes every env
    finish at step 2, so after it each env holds that step's draws (or, if it
    collided at step 1, step 1's). >= 1e6 coordinates per configuration."""
    from test_gpu_parity import make_env
    env = make_env(pkg, P, A, O, episode_len=1, seed=SEED)
    smp, _, ref_ob = reference_sample(pkg, 1 << 16, O)
    c = init_consts(smp)
    ob_init = env.obstacles.cpu().numpy().copy()
    g = torch.Generator().manual_seed(5)
    draws = [ob_init]
    steps = max(2, (2 * 1_000_000) // (P * O * 2) + 2)
    for k in range(steps):
        acts = ((torch.rand(P, A, 2, generator=g) - 0.5) * 0.8).to("cuda")
        env.step(acts)
        if k % 2 == 1:  # every env finished at this step
            draws.append(env.obstacles.cpu().numpy().copy())
    _print(f"gpu init P{P} A{A} O{O}", rs.check_obstacles(ob_init, *c, ref=ref_ob))
    fresh = np.concatenate(draws[1:])
    _print(f"gpu step re-init P{P} A{A} O{O} ({fresh.shape[0]} envs)",
           rs.check_obstacles(fresh, *c, ref=ref_ob))
    rs.check_uncorrelated(ob_init[..., 0], draws[1][..., 0], "initial vs re-init")
    assert np.count_nonzero(ob_init == draws[1]) < 1e-3 * ob_init.size


@pytest.mark.gpu
def test_gpu_native_noisy_agents_follow_reference_law(pkg):
    """Noisy native agents on the GPU (initial state and an in-step re-init)
    against the reference law."""
    from test_gpu_parity import make_env
    P = 1 << 17
    env = make_env(pkg, P, 3, 3, episode_len=1, seed=SEED, noisy_ags=True)
    smp, ref_st, _ = reference_sample(pkg, 1 << 16, 3, noisy=True)
    fm = smp.formation.numpy()
    _print("gpu noisy init", rs.check_noisy_agents(env.states.cpu().numpy(), fm, smp.ags_dist,
                                                   smp.ags_std, smp.angle_range, ref=ref_st))
    g = torch.Generator().manual_seed(6)
    for k in range(2):
        env.step(((torch.rand(P, 3, 2, generator=g) - 0.5) * 0.8).to("cuda"))
    # step 2: every env finished and re-initialised (its states are the fresh ones)
    fin = np.ones(P, bool)
    st = env.states.cpu().numpy()[fin]
    _print("gpu noisy re-init", rs.check_noisy_agents(st, fm, smp.ags_dist, smp.ags_std,
                                                      smp.angle_range, ref=ref_st))
