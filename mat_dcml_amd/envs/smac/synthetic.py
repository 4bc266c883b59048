"""SMAC-shaped synthetic battle env, vectorised on device (E envs × n_agents) — the cross-env stress config.

StarCraft II is not installable here, so BASELINE config #5 (MAT on SMAC 27m_vs_30m) runs on this stand-in
("synthetic SMAC-shaped device env"): exactly the reference's tensor contract —
``obs (E, A, 1288)``, per-agent ``state (E, A, 1458)``, ``available_actions (E, A, 36)``, per-agent dones with
dead agents inactive, episode limit 180, reward scaled by ``max_reward / 20`` and only positive
(``StarCraft2_Env.py:90-97,281-283,622-623``), ``won`` / ``battles_won`` / ``battles_game`` /
``bad_transition`` infos, auto-reset of finished episodes — with cheap kinematics instead of SC2 combat:

* allies move N/S/E/W (actions 2-5) or attack enemy j (action 6+j) within shooting range; dead allies may only
  take no-op (action 0), exactly the SMAC availability rule;
* each enemy walks to its nearest living ally and shoots it when in range;
* damage dealt, +10 per kill and +200 for the win form the (positive) reward.

It reproduces shapes, masking, episode structure and the compute of the MAT/PPO stack on SMAC, NOT SC2 dynamics:
learning-curve parity for SMAC needs a host with StarCraft II (``envs/smac/adapter.py``).

Randomness: every battle reset draws from Philox keyed by (seed, battles started, global env id, unit), so the
GPU kernel (``csrc/smac_env.hip``: the whole step + reset + observation build as ONE launch) and this torch path
produce identical battles; ``backend="auto"`` takes the kernel on a GPU.  Distances are ``sqrt(dx*dx + dy*dy)``
with every product / sum rounded separately on both paths.
"""
from __future__ import annotations

import torch

from ...utils import philox as px
from .maps import N_NO_ATTACK, SMACSpec, get_map

MAP_SIZE, SIGHT, SHOOT = 32.0, 9.0, 6.0
INV_SIGHT = 1.0 / SIGHT   # multiply by the reciprocal: torch's own tensor / scalar does, the kernel matches it
MOVE, ENEMY_MOVE = 1.0, 0.6
ALLY_DMG, ENEMY_DMG = 0.15, 0.06
DIRS = ((0.0, 1.0), (0.0, -1.0), (1.0, 0.0), (-1.0, 0.0))


class SyntheticSMACEnv:
    def __init__(self, n_envs: int, map_name: str = "27m_vs_30m", device="cpu", seed: int = 1,
                 reward_scale_rate: float = 20.0, state_per_agent: bool = True, random_agent_order: bool = False,
                 env_id_offset: int = 0, backend: str = "auto"):
        self.spec: SMACSpec = get_map(map_name)
        s = self.spec
        self.E, self.A, self.N = int(n_envs), s.n_agents, s.n_enemies
        self.n_actions = s.n_actions
        self.device = torch.device(device)
        self.k0, self.k1 = px.seed_key(int(seed))
        self.reward_scale = s.max_reward / reward_scale_rate
        self.state_per_agent = state_per_agent
        E, A, N, dev = self.E, self.A, self.N, self.device
        self.apos = torch.zeros(E, A, 2, device=dev)
        self.ahp = torch.zeros(E, A, device=dev)
        self.epos = torch.zeros(E, N, 2, device=dev)
        self.ehp = torch.zeros(E, N, device=dev)
        self.t = torch.zeros(E, dtype=torch.long, device=dev)
        self.last = torch.zeros(E, A, dtype=torch.long, device=dev)
        self.battles_won = torch.zeros(E, device=dev)
        self.battles_game = torch.zeros(E, device=dev)
        self.gid = torch.arange(E, dtype=torch.long, device=dev) + int(env_id_offset)
        self.ep_ctr = torch.zeros(E, dtype=torch.long, device=dev)   # battles started per env (reset draw counter)
        idx = torch.arange(A, device=dev)
        self.others = torch.stack([torch.cat([idx[:i], idx[i + 1:]]) for i in range(A)]) if A > 1 else \
            torch.zeros(1, 0, dtype=torch.long, device=dev)
        self.agent_id = torch.eye(A, device=dev)
        # Random_StarCraft2_Env.py:386-389: a fresh agent permutation per episode; outputs are permuted rows,
        # incoming actions are mapped back with the inverse (agent_recovery, :483-484)
        self.random_agent_order = bool(random_agent_order)
        self.perm = torch.arange(A, device=dev).expand(E, A).clone()
        self._kern = None
        if backend in ("auto", "hip") and self.device.type == "cuda":
            from ...ops import kernels
            if kernels.available() and A <= 64 and N <= 64:
                self._kern = kernels
            elif backend == "hip":
                raise RuntimeError("SMAC env kernel unavailable (HIP library not loaded or > 64 units)")

    # ------------------------------------------------------------------------------------- spaces
    @property
    def n_agents(self):
        return self.A

    @property
    def observation_space(self):
        return [[self.spec.obs_dim]] * self.A

    @property
    def share_observation_space(self):
        return [[self.spec.state_dim]] * self.A

    @property
    def action_space(self):
        return [Discrete(self.n_actions)] * self.A

    # ------------------------------------------------------------------------------------- core
    @staticmethod
    def _d2(dx, dy):
        return dx * dx + dy * dy

    def _dist(self, dx, dy):
        # fp32 squares and sum, the square root in fp64 rounded once to fp32: identical on every backend (fp32 sqrt
        # is not correctly rounded everywhere; the kernel does the same)
        return torch.sqrt((dx * dx + dy * dy).double()).float()

    def _reset_where(self, m):
        """Battle reset of the envs in ``m``: Philox draws (ep_ctr, gid, unit, P_SMAC) — ally i unit i, enemy j
        unit 64 + j; words x, y = position, z = the agent-order key (stable argsort)."""
        E, A, N, dev = self.E, self.A, self.N, self.device
        ctr, gid = self.ep_ctr.view(E, 1), self.gid.view(E, 1)
        ua = px.philox4x32(ctr, gid, torch.arange(A, device=dev).view(1, A), px.P_SMAC, self.k0, self.k1)
        ue = px.philox4x32(ctr, gid, 64 + torch.arange(N, device=dev).view(1, N), px.P_SMAC, self.k0, self.k1)

        def f(u):
            return px.u01_open(u).float()
        ap = torch.stack([8.0 + 3.0 * f(ua[0]), 16.0 + 6.0 * (f(ua[1]) - 0.5)], -1)
        ep = torch.stack([22.0 + 3.0 * f(ue[0]), 16.0 + 6.0 * (f(ue[1]) - 0.5)], -1)
        mm = m.view(E, 1)
        self.apos = torch.where(mm.unsqueeze(-1), ap, self.apos)
        self.epos = torch.where(mm.unsqueeze(-1), ep, self.epos)
        self.ahp = torch.where(mm, torch.ones_like(self.ahp), self.ahp)
        self.ehp = torch.where(mm, torch.ones_like(self.ehp), self.ehp)
        self.t = torch.where(m, torch.zeros_like(self.t), self.t)
        self.last = torch.where(mm, torch.zeros_like(self.last), self.last)
        if self.random_agent_order:
            p = torch.sort(ua[2], dim=1, stable=True).indices
            self.perm = torch.where(mm, p, self.perm)
        self.ep_ctr = torch.where(m, self.ep_ctr + 1, self.ep_ctr)

    def _rows(self, x, perm):
        if not self.random_agent_order:
            return x
        idx = perm.view(*perm.shape, *([1] * (x.dim() - 2))).expand(*perm.shape, *x.shape[2:])
        return torch.gather(x, 1, idx)

    def _observe_perm(self):
        return tuple(self._rows(x, self.perm) for x in self._observe())

    def reset(self):
        if self._kern is not None:
            return self._kern.smac_env(self, None)[:3]
        self._reset_where(torch.ones(self.E, dtype=torch.bool, device=self.device))
        return self._observe_perm()

    def step(self, actions: torch.Tensor):
        """actions (E, A[, 1]) ints.  Returns obs, state, reward (E, A, 1), dones (E, A), info dict of (E,)
        tensors, available actions."""
        E, A, N = self.E, self.A, self.N
        if self._kern is not None:   # csrc/smac_env.hip: step + battle reset + observation build in one launch
            obs, state, ava, reward, dones, info = self._kern.smac_env(self, actions)
            return obs, state, reward.view(E, 1, 1).expand(E, A, 1), dones, info, ava
        a = actions.reshape(E, A).long()
        if self.random_agent_order:   # row j of the policy output belongs to agent perm[j]
            a = torch.empty_like(a).scatter_(1, self.perm, a)
        old_perm = self.perm
        alive = self.ahp > 0
        a = torch.where(alive, a, torch.zeros_like(a))
        # moves
        dirs = torch.tensor(DIRS, device=self.device)
        mv = (a >= 2) & (a < 6)
        step = dirs[(a - 2).clamp(0, 3)] * MOVE * mv.unsqueeze(-1)
        self.apos = (self.apos + step).clamp(0.0, MAP_SIZE)
        # ally attacks
        rel = self.epos[:, None] - self.apos[:, :, None]
        d2_ae = self._d2(rel[..., 0], rel[..., 1])      # squared distances (E, A, N): range tests and the nearest
        #                                                  ally compare them, so no square root enters the dynamics
        tgt = (a - N_NO_ATTACK).clamp(0, N - 1)
        att = (a >= N_NO_ATTACK) & alive
        in_rng = torch.gather(d2_ae, 2, tgt.unsqueeze(-1)).squeeze(-1) <= SHOOT * SHOOT
        e_alive = self.ehp > 0
        hit = att & in_rng & torch.gather(e_alive, 1, tgt)
        # damage = hit count x per-hit damage (one rounding): independent of the reduction order of the scatter
        dmg = torch.zeros(E, N, device=self.device).scatter_add_(1, tgt, hit.float()) * ALLY_DMG
        old_ehp = self.ehp
        self.ehp = (self.ehp - dmg).clamp(min=0.0)
        dealt = (old_ehp - self.ehp).sum(1)
        kills = ((old_ehp > 0) & (self.ehp <= 0)).float().sum(1)
        # enemy behaviour: nearest living ally, shoot if in range else approach
        d_ea = d2_ae.transpose(1, 2).masked_fill(~alive.unsqueeze(1), float("inf"))  # (E, N, A)
        dist, near = d_ea.min(-1)                        # squared distance to the nearest living ally
        e_alive = self.ehp > 0
        shoot = e_alive & (dist <= SHOOT * SHOOT)
        walk = e_alive & (dist > SHOOT * SHOOT) & torch.isfinite(dist)
        tp = torch.gather(self.apos, 1, near.unsqueeze(-1).expand(E, N, 2))
        vec = tp - self.epos
        vec = vec / self._dist(vec[..., 0], vec[..., 1]).unsqueeze(-1).clamp(min=1e-6)
        self.epos = self.epos + vec * ENEMY_MOVE * walk.unsqueeze(-1)
        admg = torch.zeros(E, A, device=self.device).scatter_add_(1, near, shoot.float()) * ENEMY_DMG
        self.ahp = (self.ahp - admg).clamp(min=0.0)
        self.last = a
        self.t += 1
        won = (self.ehp <= 0).all(1)
        lost = (self.ahp <= 0).all(1) & ~won
        timeout = (self.t >= self.spec.limit) & ~won & ~lost
        done = won | lost | timeout
        reward = (dealt + 10.0 * kills + 200.0 * won.float()) * (1.0 / self.reward_scale)
        self.battles_game += done.float()
        self.battles_won += won.float()
        dones = (self.ahp <= 0) | done.view(E, 1)
        info = {"won": won, "lost": lost, "bad_transition": timeout, "battles_won": self.battles_won.clone(),
                "battles_game": self.battles_game.clone(), "dead_allies": (self.ahp <= 0).float().sum(1),
                "dead_enemies": (self.ehp <= 0).float().sum(1)}
        self._reset_where(done)      # unconditional: no host sync on done.any()
        obs, state, ava = self._observe_perm()
        return obs, state, reward.view(E, 1, 1).expand(E, A, 1), self._rows(dones, old_perm), info, ava

    # ------------------------------------------------------------------------------------- features
    def _observe(self):
        s, E, A, N = self.spec, self.E, self.A, self.N
        u, nA = s.unit_type_bits, self.n_actions
        dev = self.device
        alive = (self.ahp > 0).float()
        e_alive = (self.ehp > 0).float()
        last1h = torch.nn.functional.one_hot(self.last, nA).float()               # (E, A, nA)
        tb_a = torch.zeros(E, A, u, device=dev)
        if u:
            tb_a[..., 0] = 1
        # moves available: inside the map after the step
        nxt = self.apos.unsqueeze(2) + torch.tensor(DIRS, device=dev) * MOVE        # (E, A, 4, 2)
        move = (((nxt >= 0) & (nxt <= MAP_SIZE)).all(-1).float()) * alive.unsqueeze(-1)
        # enemies
        rel_e = self.epos.unsqueeze(1) - self.apos.unsqueeze(2)                      # (E, A, N, 2)
        d2_e = self._d2(rel_e[..., 0], rel_e[..., 1])
        d_e = self._dist(rel_e[..., 0], rel_e[..., 1])
        vis_e = (d2_e <= SIGHT * SIGHT).float() * e_alive.unsqueeze(1) * alive.unsqueeze(-1)
        attackable = (d2_e <= SHOOT * SHOOT).float() * vis_e
        ef = torch.stack([attackable, d_e * INV_SIGHT, rel_e[..., 0] * INV_SIGHT, rel_e[..., 1] * INV_SIGHT,
                          self.ehp.unsqueeze(1).expand(E, A, N)], -1) * vis_e.unsqueeze(-1)
        if u:
            ef = torch.cat([ef, torch.zeros(E, A, N, u, device=dev)], -1)
        # allies (others)
        oth = self.others
        rel_a = self.apos[:, oth] - self.apos.unsqueeze(2)                           # (E, A, A-1, 2)
        d_a = self._dist(rel_a[..., 0], rel_a[..., 1])
        vis_a = (self._d2(rel_a[..., 0], rel_a[..., 1]) <= SIGHT * SIGHT).float() * alive[:, oth] * alive.unsqueeze(-1)
        af = torch.cat([torch.stack([vis_a, d_a * INV_SIGHT, rel_a[..., 0] * INV_SIGHT, rel_a[..., 1] * INV_SIGHT,
                                     self.ahp[:, oth]], -1), tb_a[:, oth], last1h[:, oth]], -1) * vis_a.unsqueeze(-1)
        own = torch.cat([torch.stack([self.ahp, self.apos[..., 0] / MAP_SIZE, self.apos[..., 1] / MAP_SIZE,
                                      torch.zeros_like(self.ahp), alive], -1), tb_a, last1h], -1)
        own = own * alive.unsqueeze(-1)            # a dead unit observes nothing but its id (get_obs_agent)
        ids = self.agent_id.expand(E, A, A)
        obs = torch.cat([move, ef.reshape(E, A, -1), af.reshape(E, A, -1), own, ids], -1)
        # per-agent state: absolute positions added to every entity
        esf = torch.cat([torch.stack([attackable, d_e * INV_SIGHT, rel_e[..., 0] * INV_SIGHT, rel_e[..., 1] * INV_SIGHT,
                                      self.ehp.unsqueeze(1).expand(E, A, N),
                                      self.epos[..., 0].unsqueeze(1).expand(E, A, N) / MAP_SIZE,
                                      self.epos[..., 1].unsqueeze(1).expand(E, A, N) / MAP_SIZE,
                                      e_alive.unsqueeze(1).expand(E, A, N)], -1),
                         torch.zeros(E, A, N, u, device=dev)], -1)
        asf = torch.cat([torch.stack([vis_a, d_a * INV_SIGHT, rel_a[..., 0] * INV_SIGHT, rel_a[..., 1] * INV_SIGHT,
                                      self.ahp[:, oth], self.apos[:, oth][..., 0] / MAP_SIZE,
                                      self.apos[:, oth][..., 1] / MAP_SIZE, alive[:, oth]], -1),
                         tb_a[:, oth], last1h[:, oth]], -1)
        c = self.apos - MAP_SIZE / 2
        osf = torch.cat([torch.stack([self.ahp, self.apos[..., 0] / MAP_SIZE, self.apos[..., 1] / MAP_SIZE, alive,
                                      c[..., 0] / MAP_SIZE, c[..., 1] / MAP_SIZE, torch.zeros_like(alive)], -1),
                         tb_a, last1h], -1)
        state = torch.cat([move, esf.reshape(E, A, -1), asf.reshape(E, A, -1), osf, ids], -1)
        # availability (StarCraft2_Env.get_avail_agent_actions): dead → no-op only
        ava = torch.zeros(E, A, self.n_actions, device=dev)
        ava[..., 1] = alive
        ava[..., 2:6] = move
        ava[..., N_NO_ATTACK:] = attackable
        ava[..., 0] = 1.0 - alive
        return obs, state, ava


class Discrete:
    """Minimal ``gym.spaces.Discrete`` stand-in (gym is not a dependency); policies dispatch on the class name."""

    def __init__(self, n):
        self.n = n
        self.shape = ()
