"""ctypes wrapper of the C oracle (oracle/marlnav_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker. The product package
(marl-nav_amd/) never imports this module.

All arrays are numpy, host memory, C-contiguous; the struct types are the
ctypes mirrors of include/marlnav.h from marl-nav_amd/abi.py.
"""
import ctypes
import importlib
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
VSQRT_GRID = os.path.join(os.path.dirname(HERE), "tests", "golden", "vsqrt_r_grid.npz")
_abi = importlib.import_module("marl-nav_amd.abi")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        dims_p = ctypes.POINTER(_abi.MarlnavDims)
        par_p = ctypes.POINTER(_abi.MarlnavParams)
        lib.oracle_step.argtypes = [dims_p, par_p, ctypes.POINTER(_abi.MarlnavStepBuffers),
                                    ctypes.c_uint64, ctypes.c_int64]
        lib.oracle_step.restype = None
        lib.oracle_observe.argtypes = [dims_p, par_p, P, P, P, P]
        lib.oracle_observe.restype = None
        lib.oracle_reinit_all.argtypes = [dims_p, par_p, P, P, P, P, ctypes.c_uint64]
        lib.oracle_reinit_all.restype = None
        lib.oracle_philox2x32_10.argtypes = [P, ctypes.c_uint32, P]
        lib.oracle_philox2x32_10.restype = None
        lib.oracle_native_key.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64]
        lib.oracle_native_key.restype = ctypes.c_uint32
        lib.oracle_normalize.argtypes = [ctypes.c_int64, ctypes.c_int, P, P, P, P]
        lib.oracle_normalize.restype = None
        lib.oracle_sincos.argtypes = [ctypes.c_float, P, P]
        lib.oracle_sincos.restype = None
        lib.oracle_sincos_range.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_int, P, P]
        lib.oracle_sincos_range.restype = None
        lib.oracle_acosf_range.argtypes = [ctypes.c_uint32, ctypes.c_int64, P]
        lib.oracle_acosf_range.restype = None
        lib.oracle_set_heading_sincos.argtypes = [P, P]
        lib.oracle_set_heading_sincos.restype = None
        lib.oracle_sincos_n.argtypes = [ctypes.c_int64, P, ctypes.c_int, P, P]
        lib.oracle_sincos_n.restype = None
        lib.oracle_acosf_n.argtypes = [ctypes.c_int64, P, P]
        lib.oracle_acosf_n.restype = None
        lib.oracle_acos_device_n.argtypes = [ctypes.c_int64, P, P]
        lib.oracle_acos_device_n.restype = None
        lib.oracle_acos_device_range.argtypes = [ctypes.c_uint32, ctypes.c_int64, P]
        lib.oracle_acos_device_range.restype = None
        lib.oracle_set_acos_mode.argtypes = [ctypes.c_int]
        lib.oracle_set_acos_mode.restype = None
        lib.oracle_get_acos_mode.argtypes = []
        lib.oracle_get_acos_mode.restype = ctypes.c_int
        lib.oracle_set_vsqrt_grid.argtypes = [P, ctypes.c_int64, P, ctypes.c_int64]
        lib.oracle_set_vsqrt_grid.restype = None
        # the measured v_sqrt_f32 offsets the kernels' acos sees
        # (tests/golden/vsqrt_r_grid.npz, scripts/probes/vsqrt_grid.py): kept
        # alive here for the library's lifetime
        g = np.load(VSQRT_GRID)
        tab = (np.ascontiguousarray(g["down"], np.uint8), np.ascontiguousarray(g["up"], np.uint32))
        lib.oracle_set_vsqrt_grid(tab[0].ctypes.data, int(g["n"]), tab[1].ctypes.data, tab[1].size)
        lib._vsqrt_grid = tab
        lib.oracle_discounted_returns.argtypes = [ctypes.c_int64, ctypes.c_int64, P, P,
                                                  ctypes.c_double, P, P]
        lib.oracle_discounted_returns.restype = None
        _lib = lib
    return _lib


def _f32(a, shape=None):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    if shape is not None:
        a = a.reshape(shape)
    return a


def _ptr(a):
    return None if a is None else a.ctypes.data


def make_dims(P, A, O, S=None, env_offset=0):
    d = _abi.MarlnavDims()
    d.num_parallel, d.num_agents = int(P), int(A)
    d.obstacle_stride = int(S if S is not None else O)
    d.num_obstacles = min(int(O), d.obstacle_stride)
    d.reserved, d.env_offset = 0, int(env_offset)
    return d


def obs_dim(A, O):
    return 2 + 2 * O + 2 * (A - 1)


def observe(dims, states, obstacles, target, params=None):
    """observations() (environment.py:139-180); params supplies the angle
    cap (cap_distance; the reference's 0.1 when params is None)."""
    P, A, O = dims.num_parallel, dims.num_agents, dims.num_obstacles
    st, ob, tg = _f32(states), _f32(obstacles), _f32(target)
    out = np.empty((P, A, obs_dim(A, O)), np.float32)
    if params is None:
        params = _abi.MarlnavParams()
        params.cap_distance = 0.1
    load().oracle_observe(ctypes.byref(dims), ctypes.byref(params), _ptr(st), _ptr(ob),
                          _ptr(tg), _ptr(out))
    return out


def step(dims, params, states, obstacles, target, step_num, terminates, actions,
         fresh=None, formation=None, step_idx=0, norm=None, heading_sincos=None):
    """One Env.step on copies of the inputs. Returns a dict of outputs:
    states, obstacles, target, step_num, terminates, obs (P,A,D), reward,
    terminated, truncated, counters (trunc, col, tar), obs_norm (if norm).
    ``heading_sincos``: (sin, cos) per (env, agent) to use in the move instead
    of oracle_sincos (a test injecting the reference's own torch.sin/cos)."""
    P, A, O = dims.num_parallel, dims.num_agents, dims.num_obstacles
    D = obs_dim(A, O)
    out = {
        "states": _f32(states).copy(), "obstacles": _f32(obstacles).copy(),
        "target": _f32(target).copy(), "step_num": _f32(step_num).copy(),
        "terminates": np.ascontiguousarray(np.asarray(terminates, np.bool_)).copy(),
        "obs": np.empty((P, A, D), np.float32), "reward": np.empty(P, np.float32),
        "terminated": np.empty(P, np.bool_), "truncated": np.empty(P, np.bool_),
        "counters": np.zeros(3, np.uint64),
    }
    acts = _f32(actions)
    b = _abi.MarlnavStepBuffers()
    for k in ("states", "obstacles", "target", "step_num", "terminates", "obs",
              "reward", "terminated", "truncated", "counters"):
        setattr(b, k, _ptr(out[k]))
    b.actions = _ptr(acts)
    keep = [acts]
    if fresh is not None:
        fs, fo, ft = (_f32(x) for x in fresh)
        keep += [fs, fo, ft]
        b.fresh_states, b.fresh_obstacles, b.fresh_target = _ptr(fs), _ptr(fo), _ptr(ft)
    if formation is not None:
        fm = _f32(formation)
        keep.append(fm)
        b.formation = _ptr(fm)
    if norm is not None:
        mean, scale = _f32(norm[0]), _f32(norm[1])
        out["obs_norm"] = np.empty((P, A, D), np.float32)
        keep += [mean, scale]
        b.obs_norm, b.norm_mean, b.norm_scale = _ptr(out["obs_norm"]), _ptr(mean), _ptr(scale)
    lib = load()
    if heading_sincos is not None:
        hs, hc = (_f32(x).reshape(-1) for x in heading_sincos)
        assert hs.size == P * A and hc.size == P * A
        keep += [hs, hc]
        lib.oracle_set_heading_sincos(_ptr(hs), _ptr(hc))
    try:
        lib.oracle_step(ctypes.byref(dims), ctypes.byref(params), ctypes.byref(b),
                        int(step_idx), 1)
    finally:
        if heading_sincos is not None:
            lib.oracle_set_heading_sincos(None, None)
    out["counters"] = out["counters"].astype(np.int64)
    return out


def reinit_all(dims, params, formation, step_idx):
    P, A, S = dims.num_parallel, dims.num_agents, dims.obstacle_stride
    st = np.empty((P, A, 5), np.float32)
    ob = np.empty((P, S, 2), np.float32)
    tg = np.empty((P, 1, 2), np.float32)
    fm = _f32(formation)
    load().oracle_reinit_all(ctypes.byref(dims), ctypes.byref(params), _ptr(fm), _ptr(st),
                             _ptr(ob), _ptr(tg), int(step_idx))
    return st, ob, tg


def philox(ctr, key):
    """Philox2x32-10 of a 2-word counter under a 32-bit key (the native
    stream's generator)."""
    c = np.ascontiguousarray(ctr, np.uint32)
    o = np.empty(2, np.uint32)
    load().oracle_philox2x32_10(_ptr(c), int(key), _ptr(o))
    return o


def native_key(seed, blk, step):
    return int(load().oracle_native_key(int(seed), int(blk), int(step)))


def sincos(th, which=0):
    """oracle_sincos over an array: (sin, cos) as float32 arrays (which=1:
    the round-2 fp32 Cephes sequence, for tests/golden/libm_check.py)."""
    th = np.ascontiguousarray(th, np.float32).ravel()
    s = np.empty_like(th)
    c = np.empty_like(th)
    load().oracle_sincos_n(th.size, _ptr(th), int(which), _ptr(s), _ptr(c))
    return s, c


def acosf(x):
    """The oracle's acos (libm acosf) over an array."""
    x = np.ascontiguousarray(x, np.float32).ravel()
    out = np.empty_like(x)
    load().oracle_acosf_n(x.size, _ptr(x), _ptr(out))
    return out


def sincos_range(first_bits, n, which=0):
    """sin/cos of the n consecutive fp32 bit patterns from ``first_bits``:
    which=0 oracle_sincos (the step's), 1 the round-2 fp32 Cephes sequence
    (tests/golden/libm_check.py). The C loop runs without the GIL."""
    s = np.empty(n, np.float32)
    c = np.empty(n, np.float32)
    load().oracle_sincos_range(int(first_bits), int(n), int(which), _ptr(s), _ptr(c))
    return s, c


def acos_device(x):
    """The HIP kernel's acos (the device library's acosf, restated; its
    hardware sqrt from tests/golden/vsqrt_r_grid.npz) over an array."""
    x = np.ascontiguousarray(x, np.float32).ravel()
    out = np.empty_like(x)
    load().oracle_acos_device_n(x.size, _ptr(x), _ptr(out))
    return out


def acos_device_range(first_bits, n):
    """acos_device of n consecutive fp32 bit patterns from ``first_bits``."""
    out = np.empty(n, np.float32)
    load().oracle_acos_device_range(int(first_bits), int(n), _ptr(out))
    return out


ACOS_DEVICE, ACOS_GLIBC = 0, 1


class acos_mode:
    """Context manager / setter of the oracle's bearing acos: ACOS_DEVICE
    (default: the HIP kernel's, so kernel and oracle agree bit for bit) or
    ACOS_GLIBC (glibc acosf, the closest to the reference's MKL vsAcos)."""

    def __init__(self, mode):
        self.mode = mode
        self._saved = []

    def __enter__(self):
        lib = load()
        self._saved.append(int(lib.oracle_get_acos_mode()))  # nested uses restore in order
        lib.oracle_set_acos_mode(int(self.mode))
        return self

    def __exit__(self, *exc):
        load().oracle_set_acos_mode(self._saved.pop())
        return False


def get_acos_mode():
    return int(load().oracle_get_acos_mode())


def acosf_range(first_bits, n):
    """libm acosf (the oracle's) of n consecutive fp32 bit patterns."""
    out = np.empty(n, np.float32)
    load().oracle_acosf_range(int(first_bits), int(n), _ptr(out))
    return out


def split_obs(obs, A, O):
    """Packed (..., A, D) -> the six Observations fields (utils.py:13-15)."""
    sizes = [1, 1, O, O, A - 1, A - 1]
    edges = np.cumsum([0] + sizes)
    return [obs[..., edges[i]:edges[i + 1]] for i in range(6)]


def discounted_returns(rewards, done, gamma):
    """MAPPO._process_rewards (models.py:131-148) on (T, P) arrays: returns the
    normalized float64 returns (T, P) and (mean, std)."""
    rew = _f32(rewards)
    dn = np.ascontiguousarray(np.asarray(done, np.bool_)).view(np.uint8)
    T, P = rew.shape
    out = np.empty((T, P), np.float64)
    stats = np.empty(2, np.float64)
    load().oracle_discounted_returns(T, P, _ptr(rew), _ptr(dn), float(gamma), _ptr(out),
                                     _ptr(stats))
    return out, (float(stats[0]), float(stats[1]))
