"""Batched multi-agent particle world (MPE) on device: E worlds x N entities as tensors.

Same physics as the reference's per-object world (``mat_src/mat/envs/mpe/core.py:128-296``) but every quantity is a
tensor over (env, entity) so thousands of worlds step in a handful of fused elementwise / pairwise kernels:

* action force: ``u · accel`` for movable agents, where ``u`` was already scaled by the action sensitivity
  (``accel`` or 5.0, ``environment.py:230-234``) — the reference's double use of ``accel`` is kept;
* contact forces: for every ordered pair (i, j), i movable, both colliding:
  ``F_ij = contact_force · (p_i - p_j)/|p_i - p_j| · k · log(1 + exp(-(|p_i - p_j| - (s_i + s_j))/k))``
  (``core.py:254-279``; all masses are 1, so the mass ratio of the reference is 1);
* integration: damping, force/mass·dt, max-speed clamp, position update (``core.py:214-228``);
* communication state ``c`` = the comm action for non-silent agents, zeros for silent ones (``core.py:231-238``).

Walls (``core.py:283-296``) are not used by any reference scenario and are not modelled.
"""
from __future__ import annotations

import torch


class EntityTable:
    """Static per-entity properties (agents first, then landmarks), shared by every env of a batch."""

    def __init__(self, n_agents: int, n_landmarks: int, device, dtype=torch.float32):
        self.nA, self.nL = n_agents, n_landmarks
        n = n_agents + n_landmarks
        self.device, self.dtype = torch.device(device), dtype
        self.size = torch.full((n,), 0.05, dtype=dtype)
        self.movable = torch.zeros(n, dtype=torch.bool)
        self.movable[:n_agents] = True
        self.collide = torch.ones(n, dtype=torch.bool)
        self.accel = torch.full((n,), float("nan"), dtype=dtype)     # nan = None in the reference
        self.max_speed = torch.full((n,), float("inf"), dtype=dtype)
        self.silent = torch.zeros(n_agents, dtype=torch.bool)
        self.adversary = torch.zeros(n_agents, dtype=torch.bool)

    def finalize(self):
        for k in ("size", "movable", "collide", "accel", "max_speed", "silent", "adversary"):
            setattr(self, k, getattr(self, k).to(self.device))
        n = self.size.shape[0]
        eye = torch.eye(n, dtype=torch.bool, device=self.device)
        self.pair_min = self.size[:, None] + self.size[None, :]
        self.contact_mask = (self.collide[:, None] & self.collide[None, :] & self.movable[:, None] & ~eye)
        acc = self.accel[: self.nA]
        self.sensitivity = torch.where(torch.isnan(acc), torch.full_like(acc, 5.0), acc)
        self.force_gain = torch.where(torch.isnan(acc), torch.ones_like(acc), acc)
        return self


class World:
    """Batched world state: ``pos``/``vel`` (E, N, 2), agent comm ``c`` (E, nA, dim_c)."""

    dt, damping, contact_force, contact_margin = 0.1, 0.25, 1e2, 1e-3

    def __init__(self, n_envs: int, table: EntityTable, dim_c: int, device, dtype=torch.float32):
        self.E, self.t = int(n_envs), table
        self.dim_c, self.dim_p = dim_c, 2
        self.device, self.dtype = torch.device(device), dtype
        n = table.nA + table.nL
        self.pos = torch.zeros(self.E, n, 2, device=self.device, dtype=dtype)
        self.vel = torch.zeros_like(self.pos)
        self.c = torch.zeros(self.E, table.nA, max(dim_c, 1), device=self.device, dtype=dtype)[..., :dim_c]
        self.steps = torch.zeros(self.E, dtype=torch.long, device=self.device)

    @property
    def apos(self):
        return self.pos[:, : self.t.nA]

    @property
    def lpos(self):
        return self.pos[:, self.t.nA:]

    def collisions(self, i_idx, j_idx):
        """strict ``dist < s_i + s_j`` between entity index lists (E, len(i), len(j))"""
        d = (self.pos[:, i_idx, None, :] - self.pos[:, None, j_idx, :]).norm(dim=-1)
        return d < (self.t.size[i_idx][:, None] + self.t.size[j_idx][None, :])

    def step(self, u: torch.Tensor, comm: torch.Tensor | None):
        """``u`` (E, nA, 2) already multiplied by the sensitivity; ``comm`` (E, nA, dim_c) or None."""
        t = self.t
        nA = t.nA
        force = torch.zeros_like(self.pos)
        mov = t.movable[:nA].to(self.dtype)[None, :, None]
        force[:, :nA] = u * t.force_gain[None, :, None] * mov
        # pairwise contact forces
        delta = self.pos[:, :, None, :] - self.pos[:, None, :, :]            # (E, N, N, 2)
        dist = delta.norm(dim=-1)
        k = self.contact_margin
        pen = torch.logaddexp(torch.zeros_like(dist), -(dist - t.pair_min) / k) * k
        mask = t.contact_mask[None]
        safe = torch.where(mask, dist, torch.ones_like(dist))
        f = self.contact_force * delta / safe[..., None] * pen[..., None]
        force = force + torch.where(mask[..., None], f, torch.zeros_like(f)).sum(2)
        # integrate movable entities
        m = t.movable[None, :, None]
        vel = self.vel * (1 - self.damping) + force * self.dt
        speed = vel.norm(dim=-1, keepdim=True)
        ms = t.max_speed[None, :, None]
        vel = torch.where(speed > ms, vel / speed * ms, vel)
        self.vel = torch.where(m, vel, self.vel)
        self.pos = torch.where(m, self.pos + self.vel * self.dt, self.pos)
        if self.dim_c > 0:
            c = comm if comm is not None else torch.zeros_like(self.c)
            self.c = torch.where(t.silent[None, :, None], torch.zeros_like(c), c)
        self.steps += 1
