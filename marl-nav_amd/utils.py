"""Host-side helpers around the environment step: the Observations type, the
configuration dicts and builders the ``Env`` constructor consumes, the
initial-state and action samplers, and the observation/action transforms.

Every public name here has the name, arguments and behaviour of its
counterpart in the reference's marlnav/utils.py (cited per object), so code
written against the reference keeps working. None of it is on the per-step
compute path: ``Env.step`` runs in libmarlnav.so.
"""
import math
import random
from collections import namedtuple

import numpy as np
import torch

# utils.py:13-15 - field order is also the packed layout of include/marlnav.h
Observations = namedtuple('Observations', [
    'target_angle', 'target_distance', 'obstacles_angles',
    'obstacles_distances', 'others_angles', 'others_distances'])

# ----------------------------------------------------------------------------
# configuration dicts (utils.py:17-115). set_init_params / set_sampler_params
# update these module-level dicts in place, as the reference does.
triangle_params = {
    'init_method': 'triangle',
    'ags_cent_x': 150.0, 'ags_cent_y': 375.0, 'ags_dist': 40.0,
    'init_speed': 3.0, 'tar_pos_x': 1350.0, 'tar_pos_y': 375.0,
    'noisy_ags': False, 'ags_std': 0.01, 'angle_range': math.pi / 6,
    'obst_min_x': 500.0, 'obst_max_x': 1000.0,
    'obst_min_y': 250.0, 'obst_max_y': 500.0,
}

_SQ3 = math.sqrt(3)
# acceleration / speed-clamp scenario: 2 envs, agents heading +y
mock_params0 = {
    'init_method': 'mock_init',
    'mock_states': [[[550.0, 100.0, 0.0, 1.0, 0.0],
                     [750.0, 100.0, 0.0, 1.0, 0.0],
                     [950.0, 100.0, 0.0, 1.0, 5.0]]] * 2,
    'mock_obstacles': [[[1400.0, 375.0]]] * 2,
    'mock_target': [[[1400.0, 700.0]]] * 2,
}
# collision (env 0) and circling target-reach (env 1) scenario
mock_params1 = {
    'init_method': 'mock_init',
    'mock_states': [
        [[750.0 - 300.0 / _SQ3, 375.0, 0.0, 1.0, 3.0 / math.sin(math.pi / 3)],
         [750.0, 375.0, 0.0, 1.0, 3.0],
         [750.0 + 300.0 / _SQ3, 375.0, 0.0, 1.0, 3.0 / math.sin(math.pi / 3)]],
        [[450, 675.0, 1.0, 0.0, 2 * 300.0 * math.sin(math.radians(0.9))],
         [750.0, 675.0, 0.0, -1.0, 6.0],
         [1050.0, 675.0, -1.0, 0.0, 2 * 300.0 * math.sin(math.radians(0.9))]]],
    'mock_obstacles': [[[900.0, 475.0]], [[750.0, 75.0]]],
    'mock_target': [[[750.0, 675.0]], [[750.0, 475.0]]],
}

const_params = {'sample_method': 'const_sampler'}

sampler0_params = {
    'sampler_num': 0, 'sample_method': 'mock_sampler',
    'actions': [[[0.0, 5.0], [0.0, 0.1], [0.0, -0.05]],
                [[0.0, 5.0], [0.0, 0.1], [0.0, -100.0]]],
}
sampler1_params = {
    'sampler_num': 1, 'sample_method': 'mock_sampler',
    'actions': [[[0.0, 0.0], [0.0, 0.0], [0.0, 0.0]],
                [[-math.radians(1.8), 0.0], [0.0, 0.0], [math.radians(1.8), 0.0]]],
}


def default_args(**over):
    """The reference CLI's defaults (marlnav/__main__.py:49-132) as an
    argparse namespace, with overrides; feed it to set_env_params & co."""
    import argparse
    d = dict(seed=None, max_x_value=1500.0, max_y_value=750.0, fig_size_x=10.0,
             fig_size_y=5.0, parallel_index=0, agent_index=0, interval=10,
             random=False, weights_file=None, num_parallel=2, num_agents=3,
             num_obstacles=3, max_step=1000, episode_len=200, min_speed=3.,
             max_speed=10., min_accel=-0.5, max_accel=0.5, risk_factor=0.,
             distance_factor=0., heading_factor=500., target_factor=500.,
             soft_factor=500., bond_factor=10., hidden_size=50, learning_rate=0.001,
             ent_const=0.001, epsilon=0.01, gamma=0.9, num_total=1000000,
             buffer_len=1000, num_epochs=50, batch_size=1000, rendering=False,
             sampling_style='sampler', reward_check=False, sampler_num=-1)
    d.update(over)
    return argparse.Namespace(**d)


def _obs_bounds(num_agents, num_obstacles, max_dist):
    lo = [-math.pi, 0.0] + num_obstacles * [-math.pi] + num_obstacles * [0.0]
    lo += (num_agents - 1) * [-math.pi] + (num_agents - 1) * [0.0]
    hi = [math.pi, max_dist] + num_obstacles * [math.pi] + num_obstacles * [max_dist]
    hi += (num_agents - 1) * [math.pi] + (num_agents - 1) * [max_dist]
    return lo, hi


def set_normalizer_params(args, device):
    """utils.py:117-140: per-feature bounds of the packed observation row."""
    max_dist = math.sqrt(args.max_x_value ** 2 + args.max_y_value ** 2)
    lo, hi = _obs_bounds(args.num_agents, args.num_obstacles, max_dist)
    return {'device': device, 'num_agents': args.num_agents,
            'min_obs': lo, 'max_obs': hi}


def set_scaler_params(args, device):
    """utils.py:143-152: action bounds [-pi, pi] x [min_accel, max_accel]."""
    return {'device': device, 'num_agents': args.num_agents,
            'min_action': [-math.pi, args.min_accel],
            'max_action': [math.pi, args.max_accel]}


def set_init_params(args, device):
    """utils.py:217-232 (mutates the module dict it returns)."""
    if args.sampler_num == -1:
        p = triangle_params
        p['num_parallel'] = args.num_parallel
        p['num_obs'] = args.num_obstacles
    elif args.sampler_num == 0:
        p = mock_params0
    elif args.sampler_num == 1:
        p = mock_params1
    else:
        raise ValueError
    p['device'] = device
    return p


def set_sampler_params(args, device):
    """utils.py:235-254 (mutates the module dict it returns)."""
    if args.sampler_num == -1:
        if args.sampling_style == 'policy':
            return None
        if args.sampling_style != 'sampler':
            raise ValueError(args.sampling_style)
        p = const_params
        p['num_parallel'] = args.num_parallel
        p['num_agents'] = args.num_agents
    elif args.sampler_num in (0, 1):
        p = sampler0_params if args.sampler_num == 0 else sampler1_params
        p['max_step'] = args.max_step
    else:
        raise ValueError
    p['device'] = device
    return p


def set_env_params(args, device):
    """utils.py:257-282: the ``Env(params)`` constructor contract."""
    keys = ('num_parallel', 'num_agents', 'num_obstacles', 'max_step',
            'episode_len', 'min_speed', 'max_speed', 'min_accel', 'max_accel',
            'risk_factor', 'distance_factor', 'heading_factor', 'target_factor',
            'soft_factor', 'bond_factor')
    p = {k: getattr(args, k) for k in keys}
    p.update(device=device, x_bound=args.max_x_value, y_bound=args.max_y_value,
             sampler=set_sampler_params(args, device),
             init=set_init_params(args, device))
    return p


# ----------------------------------------------------------------- samplers
def _formation_offsets(num_agents):
    """Agent offsets (units of ags_dist/2) of the reference's 3-agent triangle
    (utils.py:349-352); for other agent counts a regular polygon with the same
    neighbour spacing (the reference has no such init: DESIGN.md §2)."""
    if num_agents == 3:
        return [[-1 / _SQ3, 1.0], [2 / _SQ3, 0.0], [-1 / _SQ3, -1.0]]
    r = 1.0 / math.sin(math.pi / num_agents)  # circumradius / (ags_dist/2)
    return [[r * math.cos(2 * math.pi * k / num_agents),
             r * math.sin(2 * math.pi * k / num_agents)] for k in range(num_agents)]


class MockInitializer(object):
    """utils.py:310-319: fixed scenario tensors, returned on every call."""

    def __init__(self, params):
        dev = params['device']
        self.states = torch.tensor(params['mock_states']).to(dev)
        self.obstacles = torch.tensor(params['mock_obstacles']).to(dev)
        self.target = torch.tensor(params['mock_target']).to(dev)

    def __call__(self):
        return self.states, self.obstacles, self.target


class TriangleIntitializer(object):
    """utils.py:322-408: formation at (ags_cent_x, ags_cent_y) heading +x,
    target at (tar_pos_x, tar_pos_y), obstacles uniform in the obstacle box.

    Host-side sampler with the reference's exact arithmetic and RNG
    consumption per call (normal_ of (P, A, 2), rand (P, A), rand (P, O, 1)
    twice), used by ``Env`` in ``rng='reference'`` mode. ``num_agents``
    defaults to the reference's hard-coded 3.
    """

    def __init__(self, params):
        self.device = params['device']
        self.init_method = params['init_method']
        self.num_parallel = params['num_parallel']
        self.num_agents = int(params.get('num_agents', 3))
        self.ags_cent_x = params['ags_cent_x']
        self.ags_cent_y = params['ags_cent_y']
        self.ags_dist = params['ags_dist']
        self.init_speed = params['init_speed']
        self.tar_pos_x = params['tar_pos_x']
        self.tar_pos_y = params['tar_pos_y']
        self.num_obs = params['num_obs']
        self.noisy_ags = int(params['noisy_ags'])
        self.ags_std = params['ags_std']
        self.angle_range = params['angle_range']
        self.obs_min_x, self.obs_max_x = params['obst_min_x'], params['obst_max_x']
        self.obs_min_y, self.obs_max_y = params['obst_min_y'], params['obst_max_y']
        self._obs_x_range = self.obs_max_x - self.obs_min_x
        self._obs_y_range = self.obs_max_y - self.obs_min_y
        self._obs_mean_x = 0.5 * (self.obs_min_x + self.obs_max_x)
        self._obs_mean_y = 0.5 * (self.obs_min_y + self.obs_max_y)
        # noise draws follow the device the reference would draw them on
        self.noise_device = params.get('noise_device', self.device)

        A, P = self.num_agents, self.num_parallel
        base = (0.5 * self.ags_dist) * torch.tensor(_formation_offsets(A))
        base = base + torch.tensor([self.ags_cent_x, self.ags_cent_y])[None, :]
        self.formation = torch.cat(
            [base, torch.tensor([[1.0, 0.0]]).repeat(A, 1),
             self.init_speed * torch.ones(A, 1)], 1)           # (A, 5) fp32
        self.target_point = torch.tensor([self.tar_pos_x, self.tar_pos_y])
        self.target = self.target_point[None, None, :].repeat(P, 1, 1).to(self.device)
        self._pos_scale = math.sqrt(self.ags_std)  # cholesky of diag(std, std)

    def __call__(self):
        states = self._sample_agents()
        obstacles = self._sample_obstacles()
        return states, obstacles, self.target

    def _sample_agents(self):
        P, A = self.num_parallel, self.num_agents
        eps = torch.empty((P, A, 2), device=self.noise_device).normal_()
        pos_noise = self.ags_dist * (self._pos_scale * eps).to('cpu')
        angles = self.noisy_ags * (self.angle_range * (torch.rand(P, A) - 0.5))
        c, s = torch.cos(angles), torch.sin(angles)
        dx, dy = self.formation[None, :, 2], self.formation[None, :, 3]
        dirs = torch.stack([c * dx + (-s) * dy, s * dx + c * dy], 2)
        pos = self.formation[None, :, :2] + self.noisy_ags * pos_noise
        speeds = self.formation[None, :, 4:5].expand(P, A, 1)
        return torch.cat([pos, dirs, speeds], 2).to(self.device)

    def _sample_obstacles(self):
        P, O = self.num_parallel, self.num_obs
        x = self._obs_x_range * (torch.rand(P, O, 1) - 0.5) + self._obs_mean_x
        y = self._obs_y_range * (torch.rand(P, O, 1) - 0.5) + self._obs_mean_y
        return torch.cat([x, y], 2).to(self.device)


def init_sampler(params):
    """utils.py:411-416"""
    if params['init_method'] == 'mock_init':
        return MockInitializer(params)
    if params['init_method'] == 'triangle':
        return TriangleIntitializer(params)
    raise NotImplementedError(params['init_method'])


class MockSampler(object):
    """utils.py:419-451: scripted actions for the mock scenarios; a generator
    that raises StopIteration after ``max_step`` calls."""

    def __init__(self, params):
        dev = params['device']
        n = params['max_step']
        env0, env1 = params['actions'][0], params['actions'][1]
        if params['sampler_num'] == 0:
            def gen():
                for _ in range(n):
                    yield torch.tensor([list(env0), list(env1)]).to(dev)
        elif params['sampler_num'] == 1:
            def gen():
                for i in range(n):
                    first = i == 0
                    row0 = [[-math.pi / 6, 0.0] if first else env0[0], env0[1],
                            [math.pi / 6, 0.0] if first else env0[2]]
                    row1 = ([[0.5 * a[0], 0.0] for a in env1] if first else list(env1))
                    yield torch.tensor([row0, row1]).to(dev)
        else:
            raise ValueError(params['sampler_num'])
        self.action_array = gen()

    def __call__(self):
        return next(self.action_array)


class ConstantSampler(object):
    """utils.py:477-485: action [0, 1] (straight ahead, full throttle)."""

    def __init__(self, params):
        self.actions = torch.tensor(
            [params['num_agents'] * [[0.0, 1.0]] for _ in range(params['num_parallel'])]
        ).to(params['device'])

    def __call__(self):
        return self.actions


def action_sampler(params):
    """utils.py:488-497"""
    if params is None:
        return None
    if params['sample_method'] == 'mock_sampler':
        return MockSampler(params)
    if params['sample_method'] == 'const_sampler':
        return ConstantSampler(params)
    raise NotImplementedError


# --------------------------------------------------------------- transforms
class ObsNormalizer(object):
    """utils.py:519-532: concatenate the Observations fields along dim 2 and
    map each feature affinely to [-1, 1]: (obs - mean) / scale.

    Observations returned by ``marlnav_amd.Env`` carry the packed (P, A, D)
    buffer they are views of; for those the concatenation is free, and when
    the env was built with this normalizer attached (``Env.attach_normalizer``)
    the kernel has already written the normalized tensor, which is returned
    as is.
    """

    def __init__(self, params):
        lo = torch.tensor(params['min_obs']).to(params['device'])
        hi = torch.tensor(params['max_obs']).to(params['device'])
        self.scale = 0.5 * (hi - lo)
        self.mean = 0.5 * (lo + hi)
        self.scale_tensor = torch.unsqueeze(torch.stack(
            [self.scale for _ in range(params['num_agents'])], dim=0), dim=0)

    def __call__(self, obs):
        pre = getattr(obs, '_normalized', None)
        if pre is not None and getattr(obs, '_normalizer', None) is self:
            return pre
        packed = getattr(obs, '_packed', None)
        x = packed if packed is not None else torch.cat(obs, dim=2)
        return (x - self.mean) / self.scale_tensor


class ActionScaler(object):
    """utils.py:535-547: actions in [-1, 1] -> scale * a + mean."""

    def __init__(self, params):
        lo = torch.tensor(params['min_action']).to(params['device'])
        hi = torch.tensor(params['max_action']).to(params['device'])
        self.scale = 0.5 * (hi - lo)
        self.mean = 0.5 * (lo + hi)
        self.scale_tensor = torch.unsqueeze(torch.stack(
            [self.scale for _ in range(params['num_agents'])], dim=0), dim=0)

    def __call__(self, actions):
        return (self.scale_tensor * actions) + self.mean


def set_all_seeds(seed):
    """utils.py:550-559"""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
        torch.backends.cudnn.deterministic = True
        torch.backends.cudnn.benchmark = False


def set_animation_params(args, device):
    """utils.py:194-214 (the keys the reward check reads: max_step,
    parallel_index, agent_index; the rest kept for callers that pass the
    dict on)."""
    return {
        'size_x': args.fig_size_x, 'size_y': args.fig_size_y,
        'x_max': args.max_x_value, 'y_max': args.max_y_value,
        'num_agents': args.num_agents, 'action_size': 2,
        'parallel_index': args.parallel_index, 'agent_index': args.agent_index,
        'sampling_style': args.sampling_style, 'random': args.random,
        'weights_file': args.weights_file, 'max_step': args.max_step,
        'interval': args.interval,
        'normalizer': set_normalizer_params(args, device),
        'scaler': set_scaler_params(args, device),
    }


CHECK_REWS_SERIES = ("target_angles", "target_distances", "all_obs_angels",
                     "all_obs_distances", "angles_to_first", "distances_to_first",
                     "angles_to_second", "distances_to_second", "rewards")


def check_rews(env, num_steps, parallel_ind, agent_ind, plot_dir='plots', plot=True):
    """utils.py:579-666: drive ``env`` with its own action sampler for
    ``num_steps`` steps and record, for env ``parallel_ind`` and agent
    ``agent_ind``, the nine series the reference plots (angle/distance to the
    target, to obstacle 0, to the first and second other agent, and the env
    reward). The series are gathered on the device and read back once (the
    reference syncs nine times per step). Saves the reference's two figures
    under ``plot_dir`` when ``plot`` (and matplotlib is importable). Returns
    {series name: list of floats} (names as in the reference, typos kept)."""
    A = env.num_agents
    others = [k for k in range(A) if k != agent_ind]
    dev = env.device
    rec = torch.empty(num_steps, 9, device=dev)
    cols = None
    for i in range(num_steps):
        actions = env.sample_actions()
        obs, rew, _, _ = env.step(actions)
        packed = getattr(obs, '_packed', None)
        if packed is None:
            packed = torch.cat(tuple(obs), dim=2)
        if cols is None:
            # observed obstacles: the obs width, which can be below
            # num_obstacles (environment.py:148-152, mock scenarios)
            O, D = obs[2].shape[-1], packed.shape[-1]
            nsec = 1 if len(others) > 1 else 0
            packed_cols = [0, 1, 2, 2 + O, 2 + 2 * O, 2 + 2 * O + (A - 1),
                           2 + 2 * O + nsec, 2 + 2 * O + (A - 1) + nsec]
            if max(packed_cols) >= D or not (0 <= parallel_ind < packed.shape[0]
                                             and 0 <= agent_ind < A):
                raise IndexError(f"check_rews: index out of range for obs {tuple(packed.shape)}")
            cols = torch.tensor(packed_cols, device=dev)
        rec[i, :8] = packed[parallel_ind, agent_ind].index_select(0, cols)
        rec[i, 8] = rew[parallel_ind]
    vals = rec.cpu().tolist()
    series = {name: [row[k] for row in vals] for k, name in enumerate(CHECK_REWS_SERIES)}
    if plot:
        _plot_check_rews(env, series, parallel_ind, agent_ind, others, plot_dir)
    return series


def _plot_check_rews(env, series, parallel_ind, agent_ind, others, plot_dir):
    """The two figures of utils.py:614-666, same titles and file names."""
    import os
    try:
        import matplotlib
        matplotlib.use('Agg')
        import matplotlib.pyplot as plt
    except ImportError:
        return
    first, second = others[0], others[1 if len(others) > 1 else 0]
    pi_plus = 3.5
    fig, axs = plt.subplots(4, 2, figsize=(10, 10))
    panels = [("target_angles", 'Angle to target (rad)', True),
              ("target_distances", 'Distance to target', False),
              ("all_obs_angels", 'Angle to obstacle (rad)', True),
              ("all_obs_distances", 'Distance to obstacle', False),
              ("angles_to_first", 'Angle to agent {} (rad)'.format(first), True),
              ("distances_to_first", 'Distance to agent {}'.format(first), False),
              ("angles_to_second", 'Angle to agent {} (rad)'.format(second), True),
              ("distances_to_second", 'Distance to agent {}'.format(second), False)]
    for ax, (key, title, is_angle) in zip(axs.flat, panels):
        ax.plot(series[key])
        ax.set_title(title)
        if is_angle:
            ax.set_ylim([-pi_plus, pi_plus])
    fig.tight_layout(pad=5.0)
    for ax in axs.flat:
        ax.set(xlabel='step number', ylabel='value')
    fig.suptitle('States, parallel index: {0}, agent index: {1}'.format(parallel_ind, agent_ind))
    os.makedirs(plot_dir, exist_ok=True)
    fig.savefig(os.path.join(plot_dir, 'states_array_{0}_agent_{1}.png'.format(
        parallel_ind, agent_ind)))
    plt.close(fig)
    fac = (env._target_factor, env._heading_factor, env._distance_factor, env._risk_factor,
           env._soft_factor, env._bond_factor)
    fig, ax = plt.subplots(1, 1)
    ax.set(xlabel='step number', ylabel='value')
    ax.plot(series["rewards"])
    fig.suptitle('Rewards, parallel index: {0}, agent index: {1}'.format(parallel_ind, agent_ind)
                 + '\n Factors: tar {0}, hea {1}'.format(fac[0], fac[1])
                 + ', dis {0}, ris {1}, sof {2} bof {3}'.format(fac[2], fac[3], fac[4], fac[5]))
    fig.savefig(os.path.join(plot_dir, 'rewards_B{0}A{1}T{2}H{3}D{4}R{5}S{6}.png'.format(
        parallel_ind, agent_ind, *fac[:5], fac[5])))
    plt.close(fig)
