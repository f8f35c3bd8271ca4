"""Faithful-structure CPU restatement of the reference's ``Env.step``.

TEST / BASELINE INFRASTRUCTURE ONLY: bench.py's ``cpu_baseline`` leg times
this module on the host cores (and, as the secondary baseline, eagerly on the
HIP device), and tests/test_torch_ref.py checks it against the golden
vectors. The product path never imports it.

It keeps the reference's execution structure (marlnav/environment.py:76-286,
utils.py:375-398), because that structure is what the baseline measures:
eager PyTorch, a nested ``vmap`` of a 2x2 rotation per agent
(environment.py:125-137), a Python loop over agents and obstacles issuing one
small cdist / normalize / einsum / acos chain per (agent, object) pair
(:139-180, 271-286), the observations computed twice per step, three
``.item()`` host reads per step (:98, 210-211) and a full-batch re-sample of
initial states every step, blended in with the int64 re-init mask by two
einsums (:76-90). The reference source itself never travels to the GPU box.
"""
import math

import torch


class TorchRefEnv:
    """Batched env; state layout as the reference's (states (P,A,5),
    obstacles (P,O,2), target (P,1,2), step_num (P,), terminates (P,))."""

    def __init__(self, P, A=3, O=3, episode_len=200, factors=None, seed=0, device="cpu",
                 bounds=None):
        self.P, self.A, self.O = P, A, O
        self.device = torch.device(device)
        self.episode_len = episode_len
        f = dict(risk=0.0, distance=0.0, heading=500.0, target=500.0, soft=500.0, bond=10.0)
        f.update(factors or {})
        self.f = f
        self.b = dict(min_speed=3.0, max_speed=10.0, min_accel=-0.5, max_accel=0.5)
        self.b.update(bounds or {})
        # geometry constants, environment.py:56-68
        self.ob_risk, self.ag_risk, self.ob_coll, self.ag_coll = 60.0, 15.0, 50.0, 5.0
        self.min_d, self.max_d, self.max_prop = 30.0, 50.0, 2
        self.max_angle, self.t_radius, self.cap = math.pi / 8, 30.0, 0.1
        self.sharp, self.ideal, self.init_dist = 1.0, 40.0, 1200.0
        self.gen = torch.Generator().manual_seed(seed)
        self.others = [torch.tensor([k for k in range(A) if k != i], device=self.device)
                       for i in range(A)]
        half = 20.0
        if A == 3:   # utils.py:350-368 formation
            offs = [[-1 / math.sqrt(3), 1.0], [2 / math.sqrt(3), 0.0], [-1 / math.sqrt(3), -1.0]]
        else:        # the build's generalised ring formation
            r = 1.0 / math.sin(math.pi / A)
            offs = [[r * math.cos(2 * math.pi * k / A), r * math.sin(2 * math.pi * k / A)]
                    for k in range(A)]
        base = half * torch.tensor(offs) + torch.tensor([150.0, 375.0])
        self.base = torch.cat([base, torch.tensor([[1.0, 0.0]]).repeat(A, 1),
                               3.0 * torch.ones(A, 1)], 1)
        self.target_init = torch.tensor([1350.0, 375.0]).view(1, 1, 2).repeat(P, 1, 1)
        self.fresh_override = None   # tests: () -> (states, obstacles, target)
        self.states, self.obstacles, self.target = self._sample()
        self.step_num = torch.zeros(P, device=self.device)
        self.terminates = torch.zeros(P, dtype=torch.bool, device=self.device)
        self.reinit_mask = torch.zeros(P, device=self.device)
        self.num_trunc = self.num_col = self.num_tar = 0

    # utils.py:375-398: one full batch per call, with the reference's draws
    def _sample(self):
        if self.fresh_override is not None:
            return tuple(t.to(self.device) for t in self.fresh_override())
        P, A, O, g = self.P, self.A, self.O, self.gen
        torch.empty(P, A, 2).normal_(generator=g)       # agent position noise (noisy_ags only)
        torch.rand(P, A, generator=g)                   # heading noise (noisy_ags only)
        xs = 500.0 * (torch.rand(P, O, 1, generator=g) - 0.5) + 750.0
        ys = 250.0 * (torch.rand(P, O, 1, generator=g) - 0.5) + 375.0
        states = self.base.unsqueeze(0).repeat(P, 1, 1)
        return (states.to(self.device), torch.cat([xs, ys], 2).to(self.device),
                self.target_init.to(self.device))

    # environment.py:286 helper chain: oriented angle to each of `others`
    @staticmethod
    def _angles(own, others, heading):
        diff = others - own.unsqueeze(1)
        unit = torch.nn.functional.normalize(diff, dim=2)
        cosang = torch.clamp(torch.einsum('pj,pkj->pk', heading, unit), -1 + 1e-8, 1 - 1e-8)
        resid = unit - torch.einsum('pk,pj->pkj', cosang, heading)
        return torch.where(resid[:, :, 0] > 0, -1.0, 1.0) * torch.acos(cosang)

    @staticmethod
    def _dists(own, others):
        return torch.cdist(own.unsqueeze(1), others)

    # environment.py:139-180: per-agent / per-obstacle loops
    def observe(self):
        st, A, O = self.states, self.A, self.O
        pos = [st[:, i, :2] for i in range(A)]
        hd = [st[:, i, 2:4] for i in range(A)]
        t_ang = torch.stack([self._angles(pos[i], self.target, hd[i]) for i in range(A)], 1)
        t_dst = torch.cat([self._dists(pos[i], self.target) for i in range(A)], 1)
        o_ang = torch.cat([torch.stack([self._angles(pos[i], self.obstacles[:, j:j + 1], hd[i])
                                        for i in range(A)], 1) for j in range(O)], 2)
        o_dst = torch.cat([torch.cat([self._dists(pos[i], self.obstacles[:, j:j + 1])
                                      for i in range(A)], 1) for j in range(O)], 2)
        nb = [torch.index_select(st, 1, self.others[i])[:, :, :2] for i in range(A)]
        a_ang = torch.stack([self._angles(pos[i], nb[i], hd[i]) for i in range(A)], 1)
        a_dst = torch.cat([self._dists(pos[i], nb[i]) for i in range(A)], 1)
        cap = self.cap
        return (torch.where(t_dst < cap, 0.0, t_ang), t_dst,
                torch.where(o_dst < cap, 0.0, o_ang), o_dst,
                torch.where(a_dst < cap, 0.0, a_ang), a_dst)

    # environment.py:236-269 helpers
    @staticmethod
    def _detect(d, radius):
        return torch.where(d < radius, 1.0, 0.0).max(dim=2)[0]

    def _distance_score(self, a_dst):
        band = torch.where(self.min_d < a_dst, 1.0, 0.0) * torch.where(a_dst < self.max_d, 1.0, 0.0)
        return torch.div(torch.clamp(band.sum(dim=2), max=self.max_prop), self.max_prop)

    def _bond(self, a_dst):
        z = (a_dst - self.ideal) / self.sharp
        return torch.mean(1.0 / (1.0 + z ** 2), dim=2)

    # environment.py:184-234
    def _rewards(self, obs):
        t_ang, t_dst, _, o_dst, _, a_dst = obs
        risk = torch.clamp(self._detect(o_dst, self.ob_risk) + self._detect(a_dst, self.ag_risk),
                           max=1)
        coll = torch.clamp(self._detect(o_dst, self.ob_coll) + self._detect(a_dst, self.ag_coll),
                           max=1)
        inside = torch.where(t_dst < self.t_radius, 1.0, 0.0)
        dist_sc = self._distance_score(a_dst)
        head = torch.where(torch.squeeze(torch.abs(t_ang), dim=2) < self.max_angle, 1.0, 0.0)
        soft = -1.0 * torch.squeeze(t_dst / self.init_dist, dim=2)
        bond = self._bond(a_dst)
        any_coll, _ = torch.max(coll, dim=1)
        all_in, _ = torch.min(inside, dim=1)
        self.num_tar += int(torch.sum(all_in).item())
        self.num_col += int(torch.sum(any_coll).item())
        terminated = torch.logical_or(any_coll > 0, self.terminates)
        self.terminates = torch.logical_and(~self.terminates, torch.squeeze(all_in) > 0)
        f = self.f
        r = (f['target'] * all_in.expand(self.P, self.A) + f['heading'] * head
             + f['distance'] * dist_sc + f['soft'] * soft + f['bond'] * bond
             - f['risk'] * risk)
        return torch.mean(r, dim=1), terminated

    # environment.py:125-137: 2x2 rotation per (env, agent) under nested vmap
    @staticmethod
    def _rotate(direction, angle):
        rot = torch.stack([torch.stack([torch.cos(angle), -torch.sin(angle)]),
                           torch.stack([torch.sin(angle), torch.cos(angle)])])
        return torch.matmul(rot, direction)

    # environment.py:113-123
    def _move(self, actions):
        th = torch.clamp(actions[:, :, 0], min=-math.pi, max=math.pi)
        self.states[:, :, 2:4] = torch.vmap(torch.vmap(self._rotate))(self.states[:, :, 2:4], th)
        acc = torch.clamp(actions[:, :, -1:], min=self.b['min_accel'], max=self.b['max_accel'])
        v = torch.clamp(self.states[:, :, 4:5] + acc, min=self.b['min_speed'],
                        max=self.b['max_speed'])
        self.states[:, :, 4:5] = v
        self.states[:, :, :2] += self.states[:, :, 2:4] * v

    # environment.py:76-90: every step, whatever the mask
    def _reinit(self):
        st, ob, tg = self._sample()
        m = self.reinit_mask

        def mix(old, new):
            return (torch.einsum('b,b...->b...', (1 - m), old)
                    + torch.einsum('b,b...->b...', m, new))
        self.states = mix(self.states, st)
        self.obstacles = mix(self.obstacles, ob)
        self.target = mix(self.target, tg)
        self.step_num = mix(self.step_num, torch.zeros(self.P, device=self.device))

    # environment.py:92-107
    def step(self, actions):
        self._move(actions)
        self.step_num += torch.ones(self.P, device=self.device)
        truncated = self.step_num > self.episode_len - 1
        self.num_trunc += torch.sum(truncated.long()).item()
        obs = self.observe()
        reward, terminated = self._rewards(obs)
        self.reinit_mask = torch.where(torch.logical_or(truncated, terminated), 1, 0)
        self._reinit()
        return self.observe(), reward, terminated, truncated
