"""Faithful-structure CPU restatement of the reference's ``Env.step``.

TEST / BASELINE INFRASTRUCTURE ONLY: bench.py's ``cpu_baseline`` leg times
this module on the host cores, and tests/test_torch_ref.py checks it against
the golden vectors. The product path never imports it.

It keeps the reference's execution structure (marlnav/environment.py:92-286,
utils.py:375-398), because that structure is what the baseline measures:
eager PyTorch on CPU, a Python loop over agents and obstacles issuing one
small cdist/normalize/einsum/acos chain per (agent, object) pair, the
observations computed twice per step, three ``.item()`` host reads per step
and a full-batch re-sample of initial states every step, blended in with the
re-init mask. The reference source itself never travels to the GPU box.
"""
import math

import torch


class TorchRefEnv:
    """Batched env on CPU tensors; state layout as the reference's."""

    def __init__(self, P, A=3, O=3, episode_len=200, factors=None, seed=0):
        self.P, self.A, self.O = P, A, O
        self.episode_len = episode_len
        f = dict(risk=0.0, distance=0.0, heading=500.0, target=500.0, soft=500.0, bond=10.0)
        f.update(factors or {})
        self.f = f
        self.bounds = dict(min_speed=3.0, max_speed=10.0, min_accel=-0.5, max_accel=0.5)
        self.gen = torch.Generator().manual_seed(seed)
        self.others = [torch.tensor([k for k in range(A) if k != i]) for i in range(A)]
        half = 20.0
        if A == 3:
            offs = [[-1 / math.sqrt(3), 1.0], [2 / math.sqrt(3), 0.0], [-1 / math.sqrt(3), -1.0]]
        else:
            r = 1.0 / math.sin(math.pi / A)
            offs = [[r * math.cos(2 * math.pi * k / A), r * math.sin(2 * math.pi * k / A)]
                    for k in range(A)]
        base = half * torch.tensor(offs) + torch.tensor([150.0, 375.0])
        self.base = torch.cat([base, torch.tensor([[1.0, 0.0]]).repeat(A, 1),
                               3.0 * torch.ones(A, 1)], 1)
        self.target_init = torch.tensor([1350.0, 375.0]).view(1, 1, 2).repeat(P, 1, 1)
        self.states, self.obstacles, self.target = self._sample()
        self.step_num = torch.zeros(P)
        self.terminates = torch.zeros(P, dtype=torch.bool)
        self.num_trunc = self.num_col = self.num_tar = 0

    # utils.py:375-398 (with the reference's RNG draws per call)
    def _sample(self):
        P, A, O, g = self.P, self.A, self.O, self.gen
        torch.empty(P, A, 2).normal_(generator=g)       # agent position noise (unused)
        torch.rand(P, A, generator=g)                   # heading noise (unused)
        xs = 500.0 * (torch.rand(P, O, 1, generator=g) - 0.5) + 750.0
        ys = 250.0 * (torch.rand(P, O, 1, generator=g) - 0.5) + 375.0
        states = self.base.unsqueeze(0).repeat(P, 1, 1)
        return states, torch.cat([xs, ys], 2), self.target_init

    # environment.py:276-286
    @staticmethod
    def _angles(own, others, heading):
        diff = others - own.unsqueeze(1)
        unit = torch.nn.functional.normalize(diff, dim=2)
        cosang = torch.clamp(torch.einsum('pj,pkj->pk', heading, unit), -1 + 1e-8, 1 - 1e-8)
        resid = unit - torch.einsum('pk,pj->pkj', cosang, heading)
        return torch.where(resid[:, :, 0] > 0, -1.0, 1.0) * torch.acos(cosang)

    # environment.py:271-274
    @staticmethod
    def _dists(own, others):
        return torch.cdist(own.unsqueeze(1), others)

    # environment.py:139-180
    def observe(self):
        st, A = self.states, self.A
        pos = [st[:, i, :2] for i in range(A)]
        hd = [st[:, i, 2:4] for i in range(A)]
        t_ang = torch.stack([self._angles(pos[i], self.target, hd[i]) for i in range(A)], 1)
        t_dst = torch.cat([self._dists(pos[i], self.target) for i in range(A)], 1)
        o_ang = torch.cat([torch.stack([self._angles(pos[i], self.obstacles[:, j:j + 1], hd[i])
                                        for i in range(A)], 1) for j in range(self.O)], 2)
        o_dst = torch.cat([torch.cat([self._dists(pos[i], self.obstacles[:, j:j + 1])
                                      for i in range(A)], 1) for j in range(self.O)], 2)
        nb = [torch.index_select(st, 1, self.others[i])[:, :, :2] for i in range(A)]
        a_ang = torch.stack([self._angles(pos[i], nb[i], hd[i]) for i in range(A)], 1)
        a_dst = torch.cat([self._dists(pos[i], nb[i]) for i in range(A)], 1)
        cap = 0.1
        return (torch.where(t_dst < cap, 0.0, t_ang), t_dst,
                torch.where(o_dst < cap, 0.0, o_ang), o_dst,
                torch.where(a_dst < cap, 0.0, a_ang), a_dst)

    # environment.py:184-269
    def _rewards(self, obs):
        t_ang, t_dst, _, o_dst, _, a_dst = obs
        hit = lambda d, r: torch.where(d < r, 1.0, 0.0).max(dim=2)[0]
        risk = torch.clamp(hit(o_dst, 60.0) + hit(a_dst, 15.0), max=1)
        coll = torch.clamp(hit(o_dst, 50.0) + hit(a_dst, 5.0), max=1)
        inside = torch.where(t_dst < 30.0, 1.0, 0.0)
        band = torch.where(30.0 < a_dst, 1.0, 0.0) * torch.where(a_dst < 50.0, 1.0, 0.0)
        dist_sc = torch.div(torch.clamp(band.sum(dim=2), max=2), 2)
        head = torch.where(torch.abs(t_ang).squeeze(2) < math.pi / 8, 1.0, 0.0)
        soft = -1.0 * torch.squeeze(t_dst / 1200.0, dim=2)
        bond = torch.mean(1.0 / (1.0 + ((a_dst - 40.0) / 1.0) ** 2), dim=2)
        any_coll, _ = coll.max(dim=1)
        all_in, _ = inside.min(dim=1)
        self.num_tar += int(all_in.sum().item())
        self.num_col += int(any_coll.sum().item())
        terminated = torch.logical_or(any_coll > 0, self.terminates)
        self.terminates = torch.logical_and(~self.terminates, all_in.squeeze() > 0)
        f = self.f
        r = (f['target'] * all_in.expand(self.P, self.A) + f['heading'] * head
             + f['distance'] * dist_sc + f['soft'] * soft + f['bond'] * bond
             - f['risk'] * risk)
        return r.mean(dim=1), terminated

    # environment.py:113-137
    def _move(self, actions):
        th = torch.clamp(actions[:, :, 0], -math.pi, math.pi)
        c, s = torch.cos(th), torch.sin(th)
        dx, dy = self.states[:, :, 2].clone(), self.states[:, :, 3].clone()
        self.states[:, :, 2] = c * dx + (-s) * dy
        self.states[:, :, 3] = s * dx + c * dy
        acc = torch.clamp(actions[:, :, -1:], self.bounds['min_accel'], self.bounds['max_accel'])
        v = torch.clamp(self.states[:, :, 4:5] + acc, self.bounds['min_speed'],
                        self.bounds['max_speed'])
        self.states[:, :, 4:5] = v
        self.states[:, :, :2] += self.states[:, :, 2:4] * v

    # environment.py:76-90
    def _blend(self, mask):
        st, ob, tg = self._sample()
        keep = 1 - mask
        mix = lambda old, new: (torch.einsum('b,b...->b...', keep, old)
                                + torch.einsum('b,b...->b...', mask, new))
        self.states = mix(self.states, st)
        self.obstacles = mix(self.obstacles, ob)
        self.target = mix(self.target, tg)
        self.step_num = mix(self.step_num, torch.zeros(self.P))

    # environment.py:92-107
    def step(self, actions):
        self._move(actions)
        self.step_num += torch.ones(self.P)
        truncated = self.step_num > self.episode_len - 1
        self.num_trunc += torch.sum(truncated.long()).item()
        obs = self.observe()
        reward, terminated = self._rewards(obs)
        mask = torch.where(torch.logical_or(truncated, terminated), 1.0, 0.0)
        self._blend(mask)
        return self.observe(), reward, terminated, truncated
