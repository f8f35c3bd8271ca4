"""Device-side rollout helpers for the training loop that drives Env.step
(SURVEY.md §8(f) row 3): MAPPO._process_rewards (marlnav/models.py:131-148)
as one HIP scan instead of a Python loop of T x 3 small tensor ops.

* ``discounted_returns(rewards, done, gamma)`` - stacked (T, P) rollout ->
  normalized float64 returns, mean, std (libmarlnav.so
  ``marlnav_discounted_returns``).
* ``process_rewards(buffer, gamma)`` - the reference's list buffer
  (``[obs, actions, log_probs, values, rewards, done]`` per step) updated in
  place exactly as ``MAPPO._process_rewards`` does; returns the mean.
* ``mappo_process_rewards(mappo)`` - drop-in body for the method (logs and
  prints like the reference).
* ``RolloutBuffer`` - preallocated stacked device storage for those six
  entries, so no per-step Python list growth and no stacking before the scan.

Numerics: float64 like the reference (its accumulator is
``torch.zeros(P, dtype=float)``); the returns recursion is evaluated in the
same order; mean and unbiased std are fixed-order two-pass reductions (torch
uses a Welford reduction), so they agree with the reference to ~1e-15
relative, not bit for bit.
"""
import ctypes

import torch

from . import abi

_F64 = torch.float64


def _stream(device):
    return torch._C._cuda_getCurrentRawStream(device.index)


def discounted_returns(rewards, done, gamma):
    """rewards (T, P) float32, done (T, P) bool, on one HIP device. Returns
    (returns (T, P) float64 normalized, mean 0-d float64, std 0-d float64)."""
    if rewards.dim() != 2 or done.shape != rewards.shape:
        raise ValueError(f"rewards and done must be (T, P); got {tuple(rewards.shape)}, "
                         f"{tuple(done.shape)}")
    dev = rewards.device
    if dev.type != "cuda":
        raise RuntimeError("discounted_returns runs on a HIP device (no CPU fallback)")
    lib = abi.load_library()
    rew = rewards.to(torch.float32).contiguous()
    dn = done.to(device=dev, dtype=torch.bool).contiguous().view(torch.uint8)
    T, P = rew.shape
    out = torch.empty(T, P, dtype=_F64, device=dev)
    stats = torch.empty(2, dtype=_F64, device=dev)
    work = torch.empty(int(lib.marlnav_returns_work_size(P)), dtype=_F64, device=dev)
    abi.check(lib.marlnav_discounted_returns(
        rew.data_ptr(), dn.data_ptr(), T, P, ctypes.c_double(float(gamma)), out.data_ptr(),
        stats.data_ptr(), work.data_ptr(), _stream(dev)), lib)
    return out, stats[0], stats[1]


def process_rewards(buffer, gamma):
    """models.py:131-148 on the reference's list buffer: every entry's reward
    slot (index -2) becomes its normalized float64 return. Returns the mean
    (0-d tensor, as the reference's ``mean_rew``)."""
    rew = torch.stack([e[-2] for e in buffer])
    done = torch.stack([e[-1] for e in buffer])
    ret, mean, _ = discounted_returns(rew, done, gamma)
    for i, e in enumerate(buffer):
        e[-2] = ret[i]
    return mean


def mappo_process_rewards(mappo):
    """Drop-in body of MAPPO._process_rewards (models.py:131-148) for a MAPPO
    instance (reads buffer, gamma; sets _mean_rew, logs and prints like the
    reference)."""
    mean = process_rewards(mappo.buffer, mappo.gamma)
    mappo._mean_rew = mean
    print('MEAN_REW', mean.item())
    mappo._logs['mean_rews'] += [mean.item()]


class RolloutBuffer(object):
    """Stacked device storage for ``buffer_len`` steps of the six rollout
    entries MAPPO.get_data keeps per step (models.py:120): obs, actions,
    log_probs, values, rewards, done. Storage is allocated on the first
    ``add`` from the shapes and dtypes given."""

    REWARDS, DONE = 4, 5

    def __init__(self, buffer_len):
        self.buffer_len = int(buffer_len)
        self._store = None
        self._n = 0
        self.returns = None

    def __len__(self):
        return self._n

    def add(self, obs, actions, log_probs, values, rewards, done):
        items = (obs, actions, log_probs, values, rewards, done)
        if self._n >= self.buffer_len:
            raise IndexError(f"rollout buffer full ({self.buffer_len} steps)")
        if self._store is None:
            self._store = [torch.empty((self.buffer_len,) + tuple(x.shape), dtype=x.dtype,
                                       device=x.device) for x in items]
        for s, x in zip(self._store, items):
            s[self._n].copy_(x)
        self._n += 1

    def clear(self):
        self._n = 0
        self.returns = None

    def stacked(self, k):
        """Entry k (0..5) of every stored step, stacked: (n, ...)."""
        return self._store[k][:self._n]

    def process_rewards(self, gamma):
        """models.py:131-148 over the stored steps; the normalized float64
        returns replace the rewards in ``entries()``. Returns the mean."""
        ret, mean, _ = discounted_returns(self.stacked(self.REWARDS), self.stacked(self.DONE),
                                          gamma)
        self.returns = ret
        return mean

    def entries(self):
        """The reference's list form: ``[[obs, actions, log_probs, values,
        reward_or_return, done], ...]`` as views of the stored steps."""
        out = []
        for t in range(self._n):
            e = [s[t] for s in self._store]
            if self.returns is not None:
                e[self.REWARDS] = self.returns[t]
            out.append(e)
        return out
