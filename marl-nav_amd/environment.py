"""Drop-in ``Env`` for marlnav/environment.py:8-286 on MI355X.

Same constructor dict, same methods (``step``, ``reset``, ``observations``,
``sample_actions``), same attributes (``states``, ``obstacles``, ``target``,
``_step_num``, ``_terminates``, ``_reinit_mask``, the episode counters
``_num_trunc/_num_col/_num_tar`` and the reward/geometry constants), same
return types and shapes. The per-step work is one launch of libmarlnav.so
(include/marlnav.h) on the current HIP stream; nothing on the step path
synchronises with the host.

Differences from the reference, all deliberate:

* ``states``/``obstacles``/``target`` are device buffers the step kernel
  writes in place. When a caller holds one (or a view), the step first moves
  the Env to a copy, so the holder sees what it would see in the reference:
  ``obstacles``/``target`` keep their pre-step values (the reference only
  rebinds them, environment.py:80-81), a held ``states`` receives the moved
  states and not the re-init (the reference moves in place, :113-123, then
  rebinds at the re-init, :79).
* The episode counters live on the device; reading one synchronises.
* ``env.step`` is the native host engine (``abi.load_host()``, C++): it
  checks the actions, picks the output tensors and enqueues the kernel
  (host side); ``Env._step_py`` handles everything the fast
  path does not (action coercion, parameter changes, reference-RNG and mock
  modes) and launches through the same engine.
* Re-initialisation randomness: ``params['rng']`` selects
  ``'native'`` (default for the triangle init: a Philox4x32-10 stream keyed
  by (seed, global env id, step), drawn on the GPU only for finished envs) or
  ``'reference'`` (the host init sampler is called every step, consuming the
  torch RNG exactly as the reference does, and finished envs take its rows).
  A user-assigned ``env._init_sampler`` is always honoured (reference mode).
"""
import ctypes
import math
import weakref

import torch

from . import abi
from .utils import MockInitializer, Observations, action_sampler, init_sampler

_F32 = torch.float32

# Env attribute -> MarlnavParams field (environment.py:32-68)
_PARAM_ATTRS = {
    'min_speed': 'min_speed', 'max_speed': 'max_speed',
    'min_accel': 'min_accel', 'max_accel': 'max_accel',
    '_risk_factor': 'risk_factor', '_distance_factor': 'distance_factor',
    '_heading_factor': 'heading_factor', '_target_factor': 'target_factor',
    '_soft_factor': 'soft_factor', '_bond_factor': 'bond_factor',
    '_ob_risk_dist': 'ob_risk_dist', '_ag_risk_dist': 'ag_risk_dist',
    '_ob_coll_dist': 'ob_coll_dist', '_ag_coll_dist': 'ag_coll_dist',
    '_agents_min_d': 'agents_min_d', '_agents_max_d': 'agents_max_d',
    '_max_at_prop_d': 'max_at_prop_d', '_max_angle_diff': 'max_angle_diff',
    '_target_radius': 'target_radius', '_cap_distance': 'cap_distance',
    '_bond_sharpness': 'bond_sharpness', '_ideal_dist': 'ideal_dist',
    '_init_dist': 'init_dist', 'episode_len': None,
}


def _f32(x):
    """Python scalar -> the fp32 value torch uses when it meets an fp32 tensor."""
    return float(torch.tensor(float(x), dtype=_F32))


# geometric constants of the reference, environment.py:56-68
GEOMETRY = {
    '_ob_risk_dist': 60., '_ag_risk_dist': 15., '_ob_coll_dist': 50.,
    '_ag_coll_dist': 5., '_agents_min_d': 30., '_agents_max_d': 50.,
    '_max_at_prop_d': 2, '_max_angle_diff': math.pi / 8, '_target_radius': 30.,
    '_cap_distance': 0.1, '_bond_sharpness': 1., '_ideal_dist': 40.,
    '_init_dist': 1200.,
}


def make_cparams(values, init=None, seed=0, flags=0):
    """Build the kernel's MarlnavParams from Env-attribute-named values
    (``min_speed``, ``_risk_factor``, ..., ``episode_len``; geometry defaults
    to GEOMETRY) and, for native re-init, the TriangleIntitializer ``init``.
    Every value is rounded to fp32 the way torch rounds a Python scalar that
    meets an fp32 tensor."""
    v = dict(GEOMETRY)
    v.update(values)
    p = abi.MarlnavParams()
    for attr, field in _PARAM_ATTRS.items():
        if field is not None:
            setattr(p, field, _f32(v[attr]))
    p.trunc_after = _f32(v['episode_len'] - 1)              # environment.py:97
    keep = flags & ~abi.NOISY_AGENTS
    if init is not None:
        p.obs_range_x = _f32(init._obs_x_range)              # utils.py:344-347
        p.obs_mean_x = _f32(init._obs_mean_x)
        p.obs_range_y = _f32(init._obs_y_range)
        p.obs_mean_y = _f32(init._obs_mean_y)
        p.ags_dist = _f32(init.ags_dist)
        p.noise_std = _f32(math.sqrt(init.ags_std))
        p.angle_range = _f32(init.angle_range)
        if init.noisy_ags:
            keep |= abi.NOISY_AGENTS
    p.flags = keep
    p.seed = int(seed) & (2 ** 64 - 1)
    return p


def _stream_handle(device):
    """Raw handle of the current HIP stream of `device` (the stream torch
    launches on; a capture stream under torch.cuda.graph)."""
    return torch._C._cuda_getCurrentRawStream(device.index)


class Env(object):
    """Parallel multi-agent navigation environment (environment.py:8)."""

    def __init__(self, params):
        object.__setattr__(self, '_params_dirty', True)
        self.params = params
        self.device = torch.device(params['device'])
        if self.device.type != 'cuda' or not torch.cuda.is_available():
            raise RuntimeError(
                "marlnav_amd.Env runs on a HIP device (params['device'] must be a "
                f"visible cuda/HIP device, got {params['device']!r}); "
                "there is no CPU fallback")
        if self.device.index is None:
            self.device = torch.device('cuda', torch.cuda.current_device())
        # params['_lib']: a loaded alternative build (scripts/graph_time.py A/B timing)
        self._lib = params.get('_lib') or abi.load_library()
        self.num_parallel = int(params['num_parallel'])
        self.num_agents = int(params['num_agents'])
        self.num_obstacles = int(params['num_obstacles'])
        self.max_step = params['max_step']
        self.episode_len = params['episode_len']
        init_p = dict(params['init'])
        if init_p.get('init_method') == 'triangle':
            init_p.setdefault('num_agents', self.num_agents)
        self._init_sampler = init_sampler(init_p)
        self._default_init_sampler = self._init_sampler
        self._sampler = action_sampler(params['sampler'])
        self._others_inds = torch.tensor(
            [[i for i in range(self.num_agents) if i != j]
             for j in range(self.num_agents)], device=self.device)

        self.min_speed = params['min_speed']
        self.max_speed = params['max_speed']
        self.min_accel = params['min_accel']
        self.max_accel = params['max_accel']
        self._risk_factor = params['risk_factor']
        self._distance_factor = params['distance_factor']
        self._heading_factor = params['heading_factor']
        self._target_factor = params['target_factor']
        self._soft_factor = params['soft_factor']
        self._bond_factor = params['bond_factor']
        for name, value in GEOMETRY.items():   # environment.py:56-68
            setattr(self, name, value)

        rng = params.get('rng', 'native')
        if rng not in ('native', 'reference'):
            raise ValueError(f"params['rng'] must be 'native' or 'reference', got {rng!r}")
        is_triangle = init_p.get('init_method') == 'triangle'
        self._rng = rng if is_triangle else 'reference'
        self._mock_alias = init_p.get('init_method') == 'mock_init'
        self._env_offset = int(params.get('env_offset', 0))
        # params['states_double_buffer']: the step reads one state buffer and
        # writes the other (MarlnavStepBuffers.states_out), the two swapping
        # roles every step; default in place (measured no faster)
        object.__setattr__(self, '_double_buffer', bool(params.get('states_double_buffer', False)))
        seed = params.get('seed', init_p.get('seed'))
        if seed is None:
            # native mode only: the reference-RNG path must not touch the torch
            # generator before the init sampler does (environment.py:26)
            seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if self._rng == 'native' else 0
        self._seed = int(seed) & (2 ** 64 - 1)
        self._normalizer = None
        self._obs_norm_buffers = None
        self._action_scaler = None
        self._engine = None

        self._dims = abi.MarlnavDims()
        self._cparams = abi.MarlnavParams()
        self._formation = None
        self._formation_obs = None
        if is_triangle:
            smp = self._init_sampler
            form = torch.cat([smp.formation.reshape(-1), smp.target_point.reshape(-1)])
            self._formation = form.to(self.device, _F32).contiguous()

        # state buffers
        P, A = self.num_parallel, self.num_agents
        if self._rng == 'native':
            S = self.num_obstacles
            self._set_state_buffers(torch.empty(P, A, 5, device=self.device),
                                    torch.empty(P, S, 2, device=self.device),
                                    torch.empty(P, 1, 2, device=self.device))
            # the fresh env's target and agent-agent pairs, observed once
            # (re-observations of finished envs then compute only obstacles)
            self._formation_obs = torch.empty(A, A, 2, device=self.device)
            abi.check(self._lib.marlnav_formation_obs(
                ctypes.byref(self._dims), self._formation.data_ptr(),
                self._formation_obs.data_ptr(), _stream_handle(self.device)), self._lib)
            self._sync_params()
            abi.check(self._lib.marlnav_reinit_all(
                ctypes.byref(self._dims), ctypes.byref(self._cparams),
                self._formation.data_ptr(), self._states.data_ptr(),
                self._obstacles.data_ptr(), self._target.data_ptr(), 0,
                _stream_handle(self.device)), self._lib)
        else:
            st, ob, tg = self._init_sampler()
            self._set_state_buffers(st, ob, tg)
        self._step_num = torch.zeros(P, device=self.device)
        self._terminates = torch.zeros(P, dtype=torch.bool, device=self.device)
        self._counters = torch.zeros(3, self._slots(), dtype=torch.int64,
                                     device=self.device)
        self._counter_out = torch.zeros(3, dtype=torch.int64, device=self.device)
        wr = weakref.ref(self)   # the engine must not keep the Env alive
        eng = abi.load_host().Engine(
            abi.fn_addr(self._lib.marlnav_step), abi.fn_addr(self._lib.marlnav_last_error),
            torch._C._cuda_getCurrentRawStream, self.device.index,
            lambda: _new_output_set(wr()), lambda a: wr()._step_py(a))
        object.__setattr__(self, '_engine', eng)
        if type(self).step is Env.step:
            # Env.step: the engine's fast path, bound on the instance. A
            # subclass that overrides step keeps its method (which reaches
            # the engine through super().step); replacing Env.step on the
            # class after construction does not reach instances already
            # built.
            object.__setattr__(self, 'step', eng)
        self._reinit_mask = torch.zeros(P, device=self.device)
        self._configure()

    # ------------------------------------------------------------ plumbing
    @property
    def allow_graph_capture(self):
        """Whether Env.step may be captured into a hipGraph (torch.cuda.graph).
        A captured step fixes the re-init draws of that call (the native RNG's
        step index, or the reference sampler's candidates), so every replay
        re-initialises finished envs identically: accepted only when set
        (timing runs such as bench.py's kernel_time_us); off by default, when
        a captured step raises."""
        return bool(self.__dict__['_engine'].allow_capture)

    @allow_graph_capture.setter
    def allow_graph_capture(self, on):
        self.__dict__['_engine'].allow_capture = 1 if on else 0

    def __setattr__(self, name, value):
        if name in _PARAM_ATTRS or name == '_init_sampler':
            object.__setattr__(self, '_params_dirty', True)
            eng = self.__dict__.get('_engine')
            if eng is not None:
                eng.fast_ok = 0   # next step goes through _step_py
        object.__setattr__(self, name, value)

    def _configure(self):
        """Push dims, parameters and the current device buffers to the host
        engine (after any of them changed)."""
        eng = self.__dict__.get('_engine')
        if eng is None:
            return
        st = self._states
        # the second states buffer (double-buffered states):
        # the engine's, unless replaced or of another shape
        alt = self.__dict__.pop('_states_alt_new', None)
        if not self.__dict__.get('_double_buffer', False):
            alt = None   # in place (the default): no second buffer at all
        else:
            if alt is None:
                alt = eng.states_alt()
            if alt is None or alt.shape != st.shape or alt.device != st.device:
                alt = torch.empty_like(st)
        b = abi.MarlnavStepBuffers()
        b.states = st.data_ptr()
        b.states_out = alt.data_ptr() if alt is not None else None
        b.obstacles = self._obstacles.data_ptr()
        b.target = self._target.data_ptr()
        b.step_num = self.__dict__['_step_num_t'].data_ptr()
        b.terminates = self.__dict__['_terminates_t'].data_ptr()
        b.counters = self._counters.data_ptr()
        b.formation = self._formation.data_ptr() if self._formation is not None else None
        fo = self.__dict__.get('_formation_obs')
        b.formation_obs = fo.data_ptr() if fo is not None else None
        if self._obs_norm_buffers is not None:
            b.norm_mean = self._obs_norm_buffers[0].data_ptr()
            b.norm_scale = self._obs_norm_buffers[1].data_ptr()
        fast = (not self._params_dirty and self._rng == 'native'
                and self._init_sampler is self._default_init_sampler)
        eng.configure(bytes(self._dims), bytes(self._cparams), bytes(b), fast)
        eng.track_state(st, self._obstacles, self._target,
                        self.__dict__['_step_num_t'], self.__dict__['_terminates_t'], alt)
        # from here the engine holds the state buffers: Env.states asks it for
        # the current one (the two swap roles every step)
        self.__dict__['_states_t'] = None
        del st, alt

    def _unshare_state(self):
        """Copy-on-write of the tensors a step writes in place. The
        reference's re-init rebinds `states`, `obstacles`, `target` and
        `_step_num` to new tensors (environment.py:79-83) and `_terminates` at
        :219, so a caller still holding one from before a step keeps its
        values - for `states` the moved ones, since `_move_agents` writes it
        in place first (:113-123), and for `_step_num` the incremented ones
        (:96, in place). The kernel writes obstacles, target, step_num and
        terminates in place and the new states into the second states buffer;
        when the engine reports one of them referenced outside the Env, the
        Env moves to a copy (stream-ordered) before the step, and a held
        second states buffer is replaced. Returns (held pre-step `states` or
        None, held pre-step `_step_num` or None) for `_finish_held`."""
        shared = self._engine.shared_state()
        held = held_sn = None
        if shared[0]:
            held = self._states
            if not self.__dict__.get('_double_buffer', False):
                # in place: the Env steps a copy
                object.__setattr__(self, '_states', held.clone())
            # double-buffered, the step reads the current buffer and writes
            # the other one, so the holder's tensor keeps its pre-step values
            # until _finish_held moves it; after the step it is the second
            # buffer, which is held and so replaced before the next step
            # (shared[5])
        if shared[5]:
            self.__dict__['_states_alt_new'] = torch.empty_like(self._states)
        if shared[1]:
            object.__setattr__(self, '_obstacles', self._obstacles.clone())
        if shared[2]:
            object.__setattr__(self, '_target', self._target.clone())
        if shared[3]:
            held_sn = self.__dict__['_step_num_t']
            self.__dict__['_step_num_t'] = held_sn.clone()
        if shared[4]:
            self.__dict__['_terminates_t'] = self.__dict__['_terminates_t'].clone()
        self._configure()
        return held, held_sn

    def _finish_held(self, held, actions_ptr):
        """What a holder of a pre-step tensor sees after the reference's step:
        the moved `states` (:113-123) and `_step_num` + 1 (:96)."""
        held_st, held_sn = held
        if held_st is not None:
            self._move_held(held_st, actions_ptr)
        if held_sn is not None:
            held_sn.add_(1.0)

    def _move_held(self, held, actions_ptr):
        """The reference's in-place `_move_agents` (environment.py:113-123) on
        a held pre-step `states` tensor: the same step kernel on that tensor
        with scratch outputs, no truncation and no collisions (trunc_after and
        the collision distances at +-inf, a zeroed `_terminates`), so no env
        finishes and the tensor receives exactly the moved states."""
        P, A = self.num_parallel, self.num_agents
        dev = self.device
        out = torch.empty(P * A * self._obs_dim + P, device=dev)
        flags = torch.zeros(3, P, dtype=torch.uint8, device=dev)
        step_num = torch.zeros(P, device=dev)
        b = abi.MarlnavStepBuffers()
        b.states = held.data_ptr()
        b.obstacles = self._obstacles.data_ptr()
        b.target = self._target.data_ptr()
        b.step_num = step_num.data_ptr()
        b.terminates = flags[2].data_ptr()
        b.actions = actions_ptr
        b.obs = out.data_ptr()
        b.reward = out[P * A * self._obs_dim:].data_ptr()
        b.terminated = flags[0].data_ptr()
        b.truncated = flags[1].data_ptr()
        # re-init sources the kernel never reads here (no env finishes)
        b.fresh_states, b.fresh_obstacles, b.fresh_target = b.states, b.obstacles, b.target
        p = abi.MarlnavParams.from_buffer_copy(self._cparams)
        p.trunc_after = float('inf')
        p.ob_coll_dist = p.ag_coll_dist = float('-inf')
        p.flags &= ~(abi.WRITE_OBS_NORM | abi.FRESH_STATES_FROM_MOVED)
        abi.check(self._lib.marlnav_step(
            ctypes.byref(self._dims), ctypes.byref(p), ctypes.byref(b),
            self._engine.step_idx, _stream_handle(dev)), self._lib)
        del out, flags, step_num   # stream-ordered: reused after the kernel

    def _slots(self):
        n = self._lib.marlnav_counter_slots(ctypes.byref(self._dims))
        if n < 0:
            abi.check(-1, self._lib)
        return n

    def _dev_f32(self, t, shape=None):
        t = torch.as_tensor(t)
        t = t.to(device=self.device, dtype=_F32).contiguous()
        if shape is not None and tuple(t.shape) != tuple(shape):
            raise ValueError(f"expected shape {tuple(shape)}, got {tuple(t.shape)}")
        return t

    def _set_state_buffers(self, states=None, obstacles=None, target=None):
        """Adopt new state tensors as the env's device buffers. Tensors that
        could alias caller storage are copied, since steps update in place."""
        P, A = self.num_parallel, self.num_agents

        def own(value, shape=None):
            t = self._dev_f32(value, shape)
            if isinstance(value, torch.Tensor) and t.data_ptr() == value.data_ptr():
                t = t.clone()
            return t

        if states is not None:
            object.__setattr__(self, '_states', own(states, (P, A, 5)))
        if obstacles is not None:
            ob = own(obstacles)
            if ob.dim() != 3 or ob.shape[0] != P or ob.shape[2] != 2:
                raise ValueError(f"obstacles must be (P, S, 2), got {tuple(ob.shape)}")
            object.__setattr__(self, '_obstacles', ob)
        if target is not None:
            object.__setattr__(self, '_target', own(target, (P, 1, 2)))
        self._update_dims()
        self._configure()

    def _update_dims(self):
        S = int(self._obstacles.shape[1])
        d = self._dims
        old = (d.num_agents, d.num_obstacles, d.obstacle_stride)
        d.num_parallel = self.num_parallel
        d.num_agents = self.num_agents
        d.num_obstacles = min(self.num_obstacles, S)   # environment.py:148-152
        d.obstacle_stride = S
        d.reserved = 0
        d.env_offset = self._env_offset
        self._obs_dim = 2 + 2 * d.num_obstacles + 2 * (self.num_agents - 1)
        self._obs_shape = (self.num_parallel, self.num_agents, self._obs_dim)
        self._act_shape = (self.num_parallel, self.num_agents, 2)
        O = d.num_obstacles
        self._split = [1, 1, O, O, self.num_agents - 1, self.num_agents - 1]
        eng = self.__dict__.get('_engine')
        if eng is not None:
            self._keep_reinit_mask()
            eng.reset_pool()               # output shapes may have changed
        if hasattr(self, '_counters') and old != (d.num_agents, d.num_obstacles, S):
            totals = self._counter_totals()
            self._counters = torch.zeros(3, self._slots(), dtype=torch.int64,
                                         device=self.device)
            self._counters[:, 0] = torch.tensor(totals, device=self.device)

    def _sync_params(self):
        if not self._params_dirty:
            return
        values = {attr: getattr(self, attr) for attr in _PARAM_ATTRS}
        init = self._default_init_sampler if self._formation is not None else None
        self._cparams = make_cparams(values, init=init, seed=self._seed,
                                     flags=self._cparams.flags & ~abi.SCALE_ACTIONS)
        if self._action_scaler is not None:
            sc = self._action_scaler
            self._cparams.act_scale[:] = [float(x) for x in sc.scale.float().reshape(-1)]
            self._cparams.act_mean[:] = [float(x) for x in sc.mean.float().reshape(-1)]
            self._cparams.flags |= abi.SCALE_ACTIONS
        object.__setattr__(self, '_params_dirty', False)
        self._configure()

    def _new_obs(self):
        return torch.empty(self.num_parallel, self.num_agents, self._obs_dim,
                           dtype=_F32, device=self.device)

    def _wrap_obs(self, packed, normalized=None):
        o = tuple.__new__(_PackedObservations, packed.split_with_sizes(self._split, 2))
        o._packed = packed
        o._normalized = normalized
        o._normalizer = self._normalizer
        return o

    # ------------------------------------------------------------ state API
    @property
    def _states(self):
        """The current states buffer: the engine's once it holds the state
        buffers (_configure), which swap roles every step (double-buffered
        states: the kernel reads one and writes the other)."""
        t = self.__dict__.get('_states_t')
        if t is not None:
            return t
        return self.__dict__['_engine'].states()

    @_states.setter
    def _states(self, t):
        self.__dict__['_states_t'] = t   # handed to the engine by _configure

    @property
    def states(self):
        return self._states

    @states.setter
    def states(self, value):
        self._set_state_buffers(states=value)

    @property
    def obstacles(self):
        return self._obstacles

    @obstacles.setter
    def obstacles(self, value):
        self._set_state_buffers(obstacles=value)

    @property
    def target(self):
        return self._target

    @target.setter
    def target(self, value):
        self._set_state_buffers(target=value)

    @property
    def _step_num(self):
        return self.__dict__['_step_num_t']

    @_step_num.setter
    def _step_num(self, value):
        t = self._dev_f32(value, (self.num_parallel,))
        if isinstance(value, torch.Tensor) and t.data_ptr() == value.data_ptr():
            t = t.clone()   # steps update it in place: never the caller's storage
        self.__dict__['_step_num_t'] = t
        self._configure()

    @property
    def _terminates(self):
        return self.__dict__['_terminates_t']

    @_terminates.setter
    def _terminates(self, value):
        t = torch.as_tensor(value).to(device=self.device, dtype=torch.bool).contiguous()
        if tuple(t.shape) != (self.num_parallel,):
            raise ValueError(f"_terminates must be ({self.num_parallel},)")
        if isinstance(value, torch.Tensor) and t.data_ptr() == value.data_ptr():
            t = t.clone()
        self.__dict__['_terminates_t'] = t
        self._configure()

    @property
    def _reinit_mask(self):
        """environment.py:102-103: set by reset(), overwritten by every step
        with where(truncated | terminated, 1, 0) (int64)."""
        eng = self._engine
        if eng.steps_done != self.__dict__.get('_reinit_mask_at'):
            last = eng.last_finished()
            if last is not None:
                term, trunc = last
                self.__dict__['_reinit_mask_t'] = torch.where(torch.logical_or(trunc, term), 1, 0)
                self.__dict__['_reinit_mask_at'] = eng.steps_done
        return self.__dict__.get('_reinit_mask_t')

    def _keep_reinit_mask(self):
        """Build `_reinit_mask` from the last step's flags before the engine
        drops its output sets (reset_pool), which hold them."""
        eng = self.__dict__.get('_engine')
        if eng is not None and eng.steps_done:
            self._reinit_mask   # noqa: B018 (materialises the cached mask)

    @_reinit_mask.setter
    def _reinit_mask(self, value):
        self.__dict__['_reinit_mask_t'] = value
        eng = self.__dict__.get('_engine')
        self.__dict__['_reinit_mask_at'] = eng.steps_done if eng is not None else None

    # episode statistics (environment.py:43-45); MAPPO reads and zeroes them
    def _counter_totals(self):
        abi.check(self._lib.marlnav_counters_total(
            ctypes.byref(self._dims), self._counters.data_ptr(),
            self._counter_out.data_ptr(), _stream_handle(self.device)), self._lib)
        return [int(v) for v in self._counter_out.tolist()]

    def _set_counter(self, row, value):
        self._counters[row].zero_()
        self._counters[row, 0] = int(value)

    @property
    def _num_trunc(self):
        return self._counter_totals()[0]

    @_num_trunc.setter
    def _num_trunc(self, v):
        self._set_counter(0, v)

    @property
    def _num_col(self):
        return self._counter_totals()[1]

    @_num_col.setter
    def _num_col(self, v):
        self._set_counter(1, v)

    @property
    def _num_tar(self):
        return self._counter_totals()[2]

    @_num_tar.setter
    def _num_tar(self, v):
        self._set_counter(2, v)

    # ----------------------------------------------------------- public API
    def attach_normalizer(self, normalizer):
        """Have every step also write ``normalizer``'s output (utils.py:519-532)
        from the kernel; ``normalizer(obs)`` then returns it without work."""
        self._normalizer = normalizer
        self._keep_reinit_mask()
        self._engine.reset_pool()
        if normalizer is None:
            self._obs_norm_buffers = None
            self._configure()
            return
        D = self._obs_dim
        mean = normalizer.mean.to(self.device, _F32).reshape(-1).contiguous()
        scale = normalizer.scale.to(self.device, _F32).reshape(-1).contiguous()
        if mean.numel() != D or scale.numel() != D:
            raise ValueError(f"normalizer has {mean.numel()} features, env rows have {D}")
        self._obs_norm_buffers = (mean, scale)
        self._configure()

    def attach_action_scaler(self, scaler):
        """Have every step read raw policy actions in [-1, 1] and apply
        ``scaler`` (an ActionScaler, utils.py:535-547) in the kernel's action
        load: ``env.step(raw)`` then equals ``env.step(scaler(raw))`` of an
        env without it. ``None`` detaches."""
        if scaler is not None and (scaler.scale.numel() != 2 or scaler.mean.numel() != 2):
            raise ValueError("ActionScaler must have 2 action components (angle, accel)")
        self._action_scaler = scaler
        object.__setattr__(self, '_params_dirty', True)
        self._engine.fast_ok = 0

    def reset(self):
        """environment.py:70-74: marks every env for re-init and returns the
        current observations (the mask is overwritten by the next step)."""
        self._reinit_mask = torch.ones(self.num_parallel, device=self.device)
        return self.observations(), self.params

    def sample_actions(self):
        """environment.py:109-111"""
        return self._sampler()

    def observations(self):
        """environment.py:139-180"""
        self._sync_params()
        out = self._new_obs()
        abi.check(self._lib.marlnav_observe(
            ctypes.byref(self._dims), ctypes.byref(self._cparams), self._states.data_ptr(),
            self._obstacles.data_ptr(), self._target.data_ptr(), out.data_ptr(),
            _stream_handle(self.device)), self._lib)
        return self._wrap_obs(out)

    def _coerce_actions(self, actions):
        actions = torch.as_tensor(actions)
        if actions.shape[-1] != 2:
            actions = actions[..., [0, -1]]  # angle = [..., 0], accel = [..., -1]
        actions = actions.to(device=self.device, dtype=_F32).contiguous()
        if actions.data_ptr() % 16:
            actions = actions.clone()   # a view at an odd offset: the compiled kernels stage 16-B pieces
        if tuple(actions.shape) != self._act_shape:
            raise ValueError(f"actions must be {self._act_shape}, got {tuple(actions.shape)}")
        return actions

    def step(self, actions):
        """environment.py:92-107: returns (Observations, rewards (P,),
        terminated (P,) bool, truncated (P,) bool). The returned tensors are
        never aliased with any tensor still referenced from a previous step;
        their memory is recycled only once nothing refers to it.

        (An Env instance's ``step`` attribute is the native host engine; this
        method is what it runs for calls its fast path does not take.)"""
        return self._engine(actions)

    def _blend_kept(self, out, fresh):
        _blend_kept_impl(self, out, fresh)

    @property
    def _step_idx(self):
        return self._engine.step_idx

    def _step_py(self, actions):
        """The step for everything the engine's fast path does not take:
        pending parameter changes, actions that need coercion (dtype, device,
        strides, a wider last axis), the reference-RNG / mock-initializer
        modes (the host init sampler is called every step, environment.py:78)."""
        if self._params_dirty:
            self._sync_params()
        held = self._unshare_state() if any(self._engine.shared_state()) else (None, None)
        dev = self.device
        if not (type(actions) is torch.Tensor and actions.dtype is _F32
                and actions.device == dev and actions.shape == self._act_shape
                and actions.is_contiguous() and not actions.requires_grad
                and actions.data_ptr() % 16 == 0):
            actions = self._coerce_actions(actions)
        eng = self._engine
        if self._rng == 'native' and self._init_sampler is self._default_init_sampler:
            if not eng.fast_ok:
                self._configure()
            out = eng.launch(actions.data_ptr(), None, 0)
            self._finish_held(held, actions.data_ptr())
            return out
        P = self.num_parallel
        fs, fo, ft = self._init_sampler()                # environment.py:78
        S = self._obstacles.shape[1]
        keep = (self._dev_f32(fs, (P, self.num_agents, 5)),
                self._dev_f32(fo, (P, S, 2)), self._dev_f32(ft, (P, 1, 2)))
        # the reference blends every env with its fresh candidate
        # (environment.py:86-90): a non-finite candidate turns even a kept
        # env's value into NaN (0 * inf). The kernel reads candidates of
        # finished envs only; kept ones are fixed up below in that case.
        poisoned = not all(bool(torch.isfinite(t).all()) for t in (fs, fo, ft))
        flags = abi.FRESH_STATES_FROM_MOVED if self._mock_alias else 0
        out = eng.launch(actions.data_ptr(), tuple(t.data_ptr() for t in keep), flags)
        if poisoned:
            self._blend_kept(out, keep)
        if self._mock_alias:
            # the reference's MockInitializer now holds the post-move states
            # (utils.py:310-319 aliasing); later re-inits restore them
            self._mock_alias = False
            init = self._init_sampler
            if isinstance(init, MockInitializer):
                init.states = self._states.clone()
        del keep   # stream-ordered: the caching allocator reuses them after the kernel
        self._finish_held(held, actions.data_ptr())
        return out


def _blend_kept_impl(env, out, fresh):
    """Kept envs (mask 0) of a step whose fresh candidates hold non-finite
    values: old + 0 * fresh (environment.py:86-90), then the step's
    observations (and the fused normaliser's copy) of the blended state,
    which for finished envs equal what the kernel wrote."""
    obs, rew, term, trunc = out
    kept = ~torch.logical_or(term, trunc)
    fs, fo, ft = fresh
    if env._mock_alias:
        fs = env._states.clone()   # the aliased mock holds the moved states
    for buf, f in ((env._states, fs), (env._obstacles, fo), (env._target, ft)):
        m = kept.view(-1, *([1] * (buf.dim() - 1)))
        buf.copy_(torch.where(m, buf + 0.0 * f, buf))
    packed = obs._packed
    abi.check(env._lib.marlnav_observe(
        ctypes.byref(env._dims), ctypes.byref(env._cparams), env._states.data_ptr(),
        env._obstacles.data_ptr(), env._target.data_ptr(), packed.data_ptr(),
        _stream_handle(env.device)), env._lib)
    if obs._normalized is not None:
        mean, scale = env._obs_norm_buffers
        torch.div(packed - mean, scale, out=obs._normalized)


def _new_output_set(env):
    """One step's output tensors carved from ONE device allocation: packed
    observations (and the fused normaliser's copy), reward, terminated,
    truncated; returns (Observations, reward, terminated, truncated, packed,
    normalized-or-None) for the host engine's pool."""
    P, A, D = env._obs_shape
    nobs = P * A * D * 4
    norm = env._obs_norm_buffers is not None

    def up(n):
        return (n + 255) & ~255
    o_norm = up(nobs)
    o_rew = o_norm + (up(nobs) if norm else 0)
    o_term = o_rew + up(4 * P)
    o_trunc = o_term + up(P)
    buf = torch.empty(o_trunc + up(P), dtype=torch.uint8, device=env.device)
    packed = buf[:nobs].view(_F32).view(P, A, D)
    normalized = buf[o_norm:o_norm + nobs].view(_F32).view(P, A, D) if norm else None
    reward = buf[o_rew:o_rew + 4 * P].view(_F32)
    terminated = buf[o_term:o_term + P].view(torch.bool)
    truncated = buf[o_trunc:o_trunc + P].view(torch.bool)
    obs = env._wrap_obs(packed, normalized)
    return obs, reward, terminated, truncated, packed, normalized


class _PackedObservations(Observations):
    """``Observations`` whose six fields are views of one packed (P, A, D)
    tensor (the layout of ObsNormalizer's torch.cat, utils.py:531); carries
    that tensor and, when a normalizer is attached, the kernel-normalized one
    (set by Env._wrap_obs)."""
