"""Generate the golden vectors that pin the oracle and the HIP path.

TEST INFRASTRUCTURE ONLY. This script runs in the build container, where the
reference (JussiM01/MARL-nav, read-only at ``$MARLNAV_REFERENCE`` or
``/root/reference``) is importable. It imports the reference's ``Env``
(marlnav/environment.py:8) unmodified, drives it, and writes inputs and
outputs as small ``.npz`` files plus ``MANIFEST.json`` next to this script.
No reference source is copied: only numbers leave the reference.

The GPU box never runs this script (``/root/reference`` does not exist
there); the committed ``.npz`` files travel instead.

Fixture classes:

* F1 ``step_*.npz``  - per-step known answers with injected state: every
  state tensor is overwritten before each ``Env.step`` and the init sampler
  is monkeypatched to return chosen fresh candidates (environment.py:76-84).
* F2 ``trace_cfg1.npz`` - the reward-check configuration
  ``python -m marlnav -rc -sn -1 -se 0`` (utils.py:579-613), 1000 steps.
* F3 ``trace_mock0.npz`` / ``trace_mock1.npz`` - the scripted mock
  scenarios ``-sn 0`` / ``-sn 1`` (utils.py:35-115, 419-451).
* F4 ``triangle_rng.npz`` - successive draws of ``TriangleIntitializer``
  after ``set_all_seeds`` (utils.py:375-398, 550-559).
* F5 ``process_rewards.npz`` - ``MAPPO._process_rewards`` (models.py:131-148)
  run unmodified (as an unbound method on a stand-in holding only the
  attributes it reads) over seeded reward/done rollouts.
* F6 ``rollout_getdata.npz`` - ``MAPPO.get_data`` (models.py:106-129) run
  unmodified on the reference's Env, with the actor and critic replaced by
  stand-ins that emit a fixed seeded action stream (the policy is not on the
  env-step path): normalised observations, raw actions, rewards, done flags
  and the processed returns of every buffer entry, plus the episode counters.

Run:  PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/make_golden.py
"""
import argparse
import json
import math
import os
import sys

os.environ.setdefault("MPLBACKEND", "Agg")
sys.dont_write_bytecode = True  # never write __pycache__ into the reference tree

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("MARLNAV_REFERENCE", "/root/reference")
sys.path.insert(0, REF)

from marlnav import utils as ref_utils  # noqa: E402
from marlnav.environment import Env as RefEnv  # noqa: E402

OBS_FIELDS = ("target_angle", "target_distance", "obstacles_angles",
              "obstacles_distances", "others_angles", "others_distances")


def cli_args(**over):
    """The reference CLI defaults (marlnav/__main__.py:49-132) as a namespace."""
    d = dict(seed=None, max_x_value=1500.0, max_y_value=750.0, fig_size_x=10.0,
             fig_size_y=5.0, parallel_index=0, agent_index=0, interval=10,
             random=False, weights_file=None, num_parallel=2, num_agents=3,
             num_obstacles=3, max_step=1000, episode_len=200, min_speed=3.,
             max_speed=10., min_accel=-0.5, max_accel=0.5, risk_factor=0.,
             distance_factor=0., heading_factor=500., target_factor=500.,
             soft_factor=500., bond_factor=10., hidden_size=50,
             learning_rate=0.001, ent_const=0.001, epsilon=0.01, gamma=0.9,
             num_total=1000000, buffer_len=1000, num_epochs=50,
             batch_size=1000, rendering=False, sampling_style='sampler',
             reward_check=True, sampler_num=-1)
    d.update(over)
    return argparse.Namespace(**d)


def ref_env(**over):
    args = cli_args(**over)
    params = ref_utils.set_params(args)
    params['env']['device'] = 'cpu'
    params['env']['init']['device'] = 'cpu'
    if params['env']['sampler'] is not None:
        params['env']['sampler']['device'] = 'cpu'
    return RefEnv(params['env']), params


def env_scalar_params(env):
    return dict(num_parallel=env.num_parallel, num_agents=env.num_agents,
                num_obstacles=env.num_obstacles, episode_len=env.episode_len,
                min_speed=env.min_speed, max_speed=env.max_speed,
                min_accel=env.min_accel, max_accel=env.max_accel,
                risk_factor=env._risk_factor, distance_factor=env._distance_factor,
                heading_factor=env._heading_factor, target_factor=env._target_factor,
                soft_factor=env._soft_factor, bond_factor=env._bond_factor)


def obs_arrays(obs):
    return {k: getattr(obs, k).detach().numpy().copy() for k in OBS_FIELDS}


# ----------------------------------------------------------------- F1 per-step
def clustered_case(gen, P, A, O):
    """Inputs built so every threshold of _rews_and_terms fires somewhere."""
    f32 = torch.float32
    cen = torch.stack([torch.rand(P, generator=gen) * 1500,
                       torch.rand(P, generator=gen) * 750], 1)
    pos = cen[:, None, :] + 18 * torch.randn(P, A, 2, generator=gen)
    ang = (torch.rand(P, A, generator=gen) - 0.5) * 2 * math.pi
    dirs = torch.stack([torch.cos(ang), torch.sin(ang)], 2)
    dirs = dirs * (0.9 + 0.2 * torch.rand(P, A, 1, generator=gen))  # drifted norms
    speed = 1.0 + 11.0 * torch.rand(P, A, 1, generator=gen)
    states = torch.cat([pos, dirs, speed], 2).to(f32)
    obstacles = (cen[:, None, :] + 55 * torch.randn(P, O, 2, generator=gen)).to(f32)
    target = (cen[:, None, :] + 25 * torch.randn(P, 1, 2, generator=gen)).to(f32)
    # edge rows: dir_y == 0 exactly, coincident agents, agent on target/obstacle
    states[0, :, 2] = 1.0
    states[0, :, 3] = 0.0
    if P > 2:
        states[1, 1, :2] = states[1, 0, :2]
        target[2, 0] = states[2, 0, :2]
        obstacles[2, 0] = states[2, 1, :2]
    if P > 4:  # whole formation inside the target area
        target[3, 0] = states[3, :, :2].mean(0)
        states[3, :, :2] = target[3, 0] + 3 * torch.randn(A, 2, generator=gen)
    return states, obstacles, target


def clustered_actions(gen, P, A, k):
    th = (torch.rand(P, A, generator=gen) - 0.5) * 9.0  # beyond +-pi: clamp
    acc = (torch.rand(P, A, generator=gen) - 0.5) * 2.5
    if k % 3 == 0:
        th[: P // 2] = 0.0  # exact straight flight on half the batch
    return torch.stack([th, acc], 2).to(torch.float32)


def make_step_case(name, P, A, O, steps, seed, factors, episode_len=20):
    gen = torch.Generator().manual_seed(seed)
    env, _ = ref_env(num_parallel=P, num_agents=A, num_obstacles=O,
                     episode_len=episode_len, **factors)
    states, obstacles, target = clustered_case(gen, P, A, O)
    step_num = torch.randint(0, episode_len + 1, (P,), generator=gen).to(torch.float32)
    terminates = torch.rand(P, generator=gen) < 0.25
    rec = {k: [] for k in (
        "in_states", "in_obstacles", "in_target", "in_step_num", "in_terminates",
        "actions", "fresh_states", "fresh_obstacles", "fresh_target",
        "out_states", "out_obstacles", "out_target", "out_step_num",
        "out_terminates", "reward", "terminated", "truncated",
        "d_trunc", "d_col", "d_tar")}
    for f in OBS_FIELDS:
        rec["obs_" + f] = []
        rec["obs0_" + f] = []
    for k in range(steps):
        fs, fo, ft = clustered_case(gen, P, A, O)
        acts = clustered_actions(gen, P, A, k)
        env.states = states.clone()
        env.obstacles = obstacles.clone()
        env.target = target.clone()
        env._step_num = step_num.clone()
        env._terminates = terminates.clone()
        env._init_sampler = (lambda fs=fs, fo=fo, ft=ft: (fs.clone(), fo.clone(), ft.clone()))
        obs0 = env.observations()  # observe-only path on the injected state
        c0 = (env._num_trunc, env._num_col, env._num_tar)
        obs, rew, term, trunc = env.step(acts.clone())
        c1 = (env._num_trunc, env._num_col, env._num_tar)
        for key, val in (("in_states", states), ("in_obstacles", obstacles),
                         ("in_target", target), ("in_step_num", step_num),
                         ("in_terminates", terminates), ("actions", acts),
                         ("fresh_states", fs), ("fresh_obstacles", fo),
                         ("fresh_target", ft), ("out_states", env.states),
                         ("out_obstacles", env.obstacles), ("out_target", env.target),
                         ("out_step_num", env._step_num),
                         ("out_terminates", env._terminates), ("reward", rew),
                         ("terminated", term), ("truncated", trunc)):
            rec[key].append(val.detach().numpy().copy())
        for f, v in obs_arrays(obs).items():
            rec["obs_" + f].append(v)
        for f, v in obs_arrays(obs0).items():
            rec["obs0_" + f].append(v)
        rec["d_trunc"].append(c1[0] - c0[0])
        rec["d_col"].append(c1[1] - c0[1])
        rec["d_tar"].append(c1[2] - c0[2])
        # chain: next step starts from the reference's own post-step state
        states, obstacles, target = env.states.clone(), env.obstacles.clone(), env.target.clone()
        step_num, terminates = env._step_num.clone(), env._terminates.clone()
    arrays = {k: np.stack(v) if not np.isscalar(v[0]) else np.asarray(v, np.int64)
              for k, v in rec.items() if v}
    arrays["in_terminates"] = arrays["in_terminates"].astype(np.bool_)
    meta = env_scalar_params(env)
    meta.update(kind="F1", steps=steps, seed=seed)
    return name, arrays, meta


# ------------------------------------------------------- F2/F3 traces
def make_trace(name, sampler_num, steps, seed):
    if seed is not None:
        ref_utils.set_all_seeds(seed)
    env, params = ref_env(sampler_num=sampler_num, max_step=steps, seed=seed)
    rec = {"states0": env.states.detach().numpy().copy(),
           "obstacles0": env.obstacles.detach().numpy().copy(),
           "target0": env.target.detach().numpy().copy()}
    seq = {k: [] for k in ("actions", "states", "obstacles", "target", "reward",
                           "terminated", "truncated", "num_trunc", "num_col",
                           "num_tar", "step_num", "terminates")}
    for f in OBS_FIELDS:
        seq["obs_" + f] = []
    for _ in range(steps):
        acts = env.sample_actions()
        seq["actions"].append(acts.detach().numpy().copy())
        obs, rew, term, trunc = env.step(acts)
        for f, v in obs_arrays(obs).items():
            seq["obs_" + f].append(v)
        seq["reward"].append(rew.numpy().copy())
        seq["terminated"].append(term.numpy().copy())
        seq["truncated"].append(trunc.numpy().copy())
        seq["states"].append(env.states.detach().numpy().copy())
        seq["obstacles"].append(env.obstacles.detach().numpy().copy())
        seq["target"].append(env.target.detach().numpy().copy())
        seq["step_num"].append(env._step_num.numpy().copy())
        seq["terminates"].append(env._terminates.numpy().copy())
        seq["num_trunc"].append(env._num_trunc)
        seq["num_col"].append(env._num_col)
        seq["num_tar"].append(env._num_tar)
    rec.update({k: np.asarray(v) for k, v in seq.items()})
    meta = env_scalar_params(env)
    meta.update(kind="trace", sampler_num=sampler_num, steps=steps, seed=seed,
                init=params['env']['init']['init_method'])
    return name, rec, meta


# ----------------------------------------------------------------- F4 RNG
def make_triangle_rng(seeds=(0, 1, 7), P=8, O=3, draws=4):
    rec, meta = {}, {"kind": "F4", "num_parallel": P, "num_obstacles": O,
                     "draws": draws, "seeds": list(seeds)}
    for s in seeds:
        ref_utils.set_all_seeds(s)
        args = cli_args(num_parallel=P, num_obstacles=O)
        init = ref_utils.init_sampler(ref_utils.set_init_params(args, 'cpu'))
        st, ob, tg = [], [], []
        for _ in range(draws):
            a, b, c = init()
            st.append(a.numpy().copy()); ob.append(b.numpy().copy()); tg.append(c.numpy().copy())
        rec[f"seed{s}_states"] = np.stack(st)
        rec[f"seed{s}_obstacles"] = np.stack(ob)
        rec[f"seed{s}_target"] = np.stack(tg)
    return "triangle_rng", rec, meta


# ------------------------------------------------------- F5 process_rewards
class _RolloutHolder(object):
    """The attributes MAPPO._process_rewards reads and writes."""


def make_process_rewards(cases=((24, 96, 0.9, 21, 0.1), (7, 5, 0.99, 22, 0.3),
                                (1, 33, 0.9, 23, 0.0))):
    from marlnav.models import MAPPO
    rec, meta = {}, {"kind": "F5", "cases": []}
    for k, (T, P, gamma, seed, p_done) in enumerate(cases):
        g = torch.Generator().manual_seed(seed)
        rew = (torch.randn(T, P, generator=g) * 200.0).to(torch.float32)
        done = torch.rand(T, P, generator=g) < p_done
        h = _RolloutHolder()
        h.buffer = [[None, None, None, None, rew[t].clone(), done[t].clone()] for t in range(T)]
        h.buffer_len, h.num_parallel, h.device, h.gamma = T, P, "cpu", gamma
        h._logs = {"mean_rews": []}
        h._mean_rew = 0.0
        MAPPO._process_rewards(h)
        rec[f"case{k}_rewards"] = rew.numpy()
        rec[f"case{k}_done"] = done.numpy()
        rec[f"case{k}_returns"] = np.stack([h.buffer[t][-2].numpy() for t in range(T)])
        rec[f"case{k}_mean"] = np.float64(h._mean_rew.item())
        meta["cases"].append({"T": T, "P": P, "gamma": gamma, "seed": seed, "p_done": p_done,
                              "returns_dtype": str(h.buffer[0][-2].dtype)})
    return "process_rewards", rec, meta


# ------------------------------------------------------- F6 MAPPO get_data
class _FixedActor(torch.nn.Module):
    """Actor stand-in: the next (P*A, 2) block of a fixed action stream as a
    'distribution' (sample / log_prob), like models.py:113-115 expects."""

    def __init__(self, stream):
        super().__init__()
        self.stream = stream
        self.t = 0

    def forward(self, obs):
        a = self.stream[self.t]
        self.t += 1

        class _Dist:
            def sample(self):
                return a.clone()

            def log_prob(self, x):
                return torch.zeros(x.shape[0])
        return _Dist()


class _ZeroCritic(torch.nn.Module):
    def forward(self, obs):
        return torch.zeros(obs.shape[0], 1)


def make_rollout(P=24, T=200, episode_len=40, seed=5, action_seed=31, gamma=0.9):
    import contextlib
    import io
    import tempfile
    from marlnav.models import MAPPO
    args = cli_args(num_parallel=P, episode_len=episode_len, buffer_len=T, batch_size=T,
                    num_total=P * T, gamma=gamma, reward_check=False, seed=seed,
                    risk_factor=3.0, distance_factor=7.0)
    ref_utils.set_all_seeds(seed)
    params = ref_utils.set_params(args)
    for k in ("env", "model"):
        params[k]['device'] = 'cpu'
    params['env']['init']['device'] = 'cpu'
    params['model']['normalizer']['device'] = 'cpu'
    params['model']['scaler']['device'] = 'cpu'
    env = RefEnv(params['env'])
    g = torch.Generator().manual_seed(action_seed)
    stream = [(torch.rand(P * 3, 2, generator=g) * 2.4 - 1.2) for _ in range(T)]
    rec = {"states0": env.states.numpy().copy(), "obstacles0": env.obstacles.numpy().copy()}
    raw = {"reward": [], "terminated": [], "truncated": []}
    step = env.step

    def recording_step(actions):
        out = step(actions)
        raw["reward"].append(out[1].numpy().copy())
        raw["terminated"].append(out[2].numpy().copy())
        raw["truncated"].append(out[3].numpy().copy())
        return out
    env.step = recording_step
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                model = MAPPO(params['model'], env)
                model.actor = _FixedActor(stream)
                model.critic = _ZeroCritic()
                ref_utils.set_all_seeds(seed + 1)   # the env's draws from here on
                model.get_data()
        finally:
            os.chdir(cwd)
    rec["actions"] = torch.stack(stream).numpy()
    rec["obs_norm"] = np.stack([model.buffer[t][0].numpy() for t in range(T)])
    rec["done"] = np.stack([model.buffer[t][5].numpy() for t in range(T)])
    rec["returns"] = np.stack([model.buffer[t][4].numpy() for t in range(T)])
    rec["final_obs_norm"] = model.obs.numpy()
    for k, v in raw.items():
        rec[k] = np.stack(v)
    rec["mean_rew"] = np.float64(model._mean_rew.item())
    stats = model._logs['epi_stats']
    meta = {"kind": "F6", "num_parallel": P, "buffer_len": T, "episode_len": episode_len,
            "seed": seed, "reseed": seed + 1, "action_seed": action_seed, "gamma": gamma,
            "risk_factor": 3.0, "distance_factor": 7.0,
            "action_stream": "torch.rand(P*3, 2, Generator(action_seed)) * 2.4 - 1.2 per step",
            "num_trunc": stats['trunc'][-1], "num_col": stats['col'][-1],
            "num_tar": stats['tar'][-1], "returns_dtype": str(model.buffer[0][4].dtype)}
    return "rollout_getdata", rec, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", help="fixture names to (re)generate")
    cli = ap.parse_args()
    torch.set_num_threads(1)
    all_factors = dict(risk_factor=3., distance_factor=7., heading_factor=500.,
                       target_factor=500., soft_factor=500., bond_factor=10.)
    jobs = [
        make_step_case("step_a3o3", 64, 3, 3, 8, 11, all_factors),
        make_step_case("step_a3o8", 64, 3, 8, 6, 12, all_factors),
        make_step_case("step_a16o32", 16, 16, 32, 4, 13, all_factors),
        make_step_case("step_a2o1", 32, 2, 1, 6, 14, all_factors),
        make_step_case("step_p1", 1, 3, 3, 12, 15, all_factors, episode_len=5),
        make_trace("trace_cfg1", -1, 1000, 0),
        make_trace("trace_mock0", 0, 1000, None),
        make_trace("trace_mock1", 1, 1000, None),
        make_triangle_rng(),
        make_process_rewards(),
        make_rollout(),
    ] if not cli.only else [JOBS[n]() for n in cli.only]
    mpath = os.path.join(HERE, "MANIFEST.json")
    manifest = {"torch": torch.__version__, "numpy": np.__version__,
                "cpu_capability": torch.backends.cpu.get_cpu_capability(),
                "reference": "JussiM01/MARL-nav @ 2025-10-03 (imported unmodified)",
                "generator": "tests/golden/make_golden.py", "files": {}}
    if os.path.exists(mpath):
        with open(mpath) as fh:
            old = json.load(fh)
        # entries other scripts own (tests/golden/libm_check.py: "libm")
        for k, v in old.items():
            manifest.setdefault(k, v)
        if cli.only:
            manifest["files"] = old["files"]
    for name, arrays, meta in jobs:
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **arrays)
        manifest["files"][name + ".npz"] = meta
        print(f"{name}: {os.path.getsize(path)} bytes")
    with open(mpath, "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)


JOBS = {"process_rewards": make_process_rewards, "triangle_rng": make_triangle_rng,
        "rollout_getdata": make_rollout}


if __name__ == "__main__":
    main()
