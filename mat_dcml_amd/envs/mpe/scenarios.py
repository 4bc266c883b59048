"""The reference's nine MPE scenarios as batched tensor programs (``mat_src/mat/envs/mpe/scenarios/*.py``).

Each scenario owns its per-env episode variables (goals, keys, colours) as (E, ...) tensors and provides
``make`` (entity table), ``reset(world, mask)`` (resample the masked envs), ``observation(world)`` (list of
per-agent (E, d_i) tensors, the reference's concatenation order), ``reward(world)`` (E, nA) and ``info``.

Reference quirks kept on purpose (each is what the reference computes):
* ``simple_spread``: an agent counts itself as a collision (``is_collision(a, agent)`` over all agents includes
  ``a is agent``, dist 0 < 2·size), so every agent gets an extra -1 each step (``simple_spread.py:89-92``).
* ``simple_tag`` / ``simple_world_comm``: adversaries are rewarded for EVERY (good, adversary) collision pair, not
  only their own (``simple_tag.py:118-121``).
* ``simple_world_comm``: all landmarks (obstacles, food, forests) are placed once and food / forests are then
  placed again (``simple_world_comm.py:102-110``); boundaries are never added (``set_boundaries`` is unused).
* ``simple_attack``: the reference module calls ``bound`` as a free function that only exists as an unbound
  method, so its reward raises ``NameError`` (``simple_attack.py:68-73,92``).  The intended bound penalty is used
  here; ``info['fail']`` becomes True after the first good-agent reward, as in the reference (``:88``).
"""
from __future__ import annotations

import torch

from .core import EntityTable, World


def _u(gen, E, n, device, dtype, scale=1.0):
    return scale * (2.0 * torch.rand(E, n, 2, generator=gen, device=device, dtype=dtype) - 1.0)


def _choice(gen, E, n, device):
    return torch.randint(0, n, (E,), generator=gen, device=device)


def _bound(x):
    """per-coordinate boundary penalty of simple_tag / simple_world_comm (``simple_tag.py:99-104``)"""
    return torch.where(x < 0.9, torch.zeros_like(x),
                       torch.where(x < 1.0, (x - 0.9) * 10, torch.clamp(torch.exp(2 * x - 2), max=10.0)))


def _gather_rows(x, idx):
    """x (E, N, D), idx (E,) -> (E, D)"""
    return x[torch.arange(x.shape[0], device=x.device), idx]


class Scenario:
    name = ""
    collaborative = False
    world_length = 25
    dim_c = 0

    def __init__(self, args):
        self.args = args

    # per-agent action heads: (movable: 5-way move, comm: dim_c-way message or 0)
    def heads(self, t: EntityTable):
        return [(bool(t.movable[i]), 0 if bool(t.silent[i]) else self.dim_c) for i in range(t.nA)]

    def info(self, w: World):
        return {}

    def _place(self, w, mask, gen, agent_scale=1.0, landmark_scale=0.8):
        E, dev, dt = w.E, w.device, w.dtype
        nA, nL = w.t.nA, w.t.nL
        p = torch.cat([_u(gen, E, nA, dev, dt, agent_scale), _u(gen, E, nL, dev, dt, landmark_scale)], 1)
        m = mask[:, None, None]
        w.pos = torch.where(m, p, w.pos)
        w.vel = torch.where(m, torch.zeros_like(w.vel), w.vel)
        if w.dim_c:
            w.c = torch.where(m, torch.zeros_like(w.c), w.c)


class SimpleSpread(Scenario):
    name, collaborative, dim_c = "simple_spread", True, 2

    def make(self, args):
        self.world_length = args.episode_length
        t = EntityTable(args.num_agents, args.num_landmarks, "cpu")
        t.size[: t.nA] = 0.15
        t.silent[:] = True
        t.collide[t.nA:] = False
        t.movable[t.nA:] = False
        return t

    def reset(self, w, mask, gen):
        self._place(w, mask, gen)

    def observation(self, w):
        nA = w.t.nA
        ap, av, lp = w.apos, w.vel[:, :nA], w.lpos
        out = []
        for i in range(nA):
            others = [j for j in range(nA) if j != i]
            parts = [av[:, i], ap[:, i], (lp - ap[:, i: i + 1]).flatten(1), (ap[:, others] - ap[:, i: i + 1]).flatten(1),
                     w.c[:, others].flatten(1)]
            out.append(torch.cat(parts, 1))
        return out

    def reward(self, w):
        nA = w.t.nA
        d = (w.apos[:, :, None] - w.lpos[:, None]).norm(dim=-1)       # (E, nA, nL)
        cover = -d.min(1).values.sum(1, keepdim=True)                   # (E, 1)
        col = w.collisions(list(range(nA)), list(range(nA))).sum(2).to(w.dtype)   # includes self
        return cover - col


class SimpleReference(Scenario):
    name, collaborative, dim_c = "simple_reference", True, 10
    LCOL = ((0.75, 0.25, 0.25), (0.25, 0.75, 0.25), (0.25, 0.25, 0.75))

    def make(self, args):
        assert args.num_agents == 2, "only 2 agents is supported"
        self.world_length = args.episode_length
        t = EntityTable(2, args.num_landmarks, "cpu")
        t.collide[:] = False
        t.movable[2:] = False
        return t

    def reset(self, w, mask, gen):
        if not hasattr(self, "goal_b"):
            self.goal_b = torch.zeros(w.E, 2, dtype=torch.long, device=w.device)
            self.lcol = torch.tensor(self.LCOL, dtype=w.dtype, device=w.device)[: w.t.nL]
        g = torch.stack([_choice(gen, w.E, w.t.nL, w.device), _choice(gen, w.E, w.t.nL, w.device)], 1)
        self.goal_b = torch.where(mask[:, None], g, self.goal_b)
        self._place(w, mask, gen)

    def observation(self, w):
        ap, av, lp = w.apos, w.vel[:, :2], w.lpos
        out = []
        for i in range(2):
            col = self.lcol[self.goal_b[:, i]]
            out.append(torch.cat([av[:, i], (lp - ap[:, i: i + 1]).flatten(1), col, w.c[:, 1 - i]], 1))
        return out

    def reward(self, w):
        r = []
        for i in range(2):
            gl = _gather_rows(w.lpos, self.goal_b[:, i])
            r.append(-((w.apos[:, 1 - i] - gl) ** 2).sum(1))
        return torch.stack(r, 1)


class SimpleSpeakerListener(Scenario):
    name, collaborative, dim_c = "simple_speaker_listener", True, 3
    LCOL = ((0.65, 0.15, 0.15), (0.15, 0.65, 0.15), (0.15, 0.15, 0.65))

    def make(self, args):
        assert args.num_agents == 2, "only 2 agents is supported"
        self.world_length = args.episode_length
        t = EntityTable(2, args.num_landmarks, "cpu")
        t.collide[:] = False
        t.size[:2] = 0.075
        t.size[2:] = 0.04
        t.movable[0] = False
        t.movable[2:] = False
        t.silent[1] = True
        return t

    def reset(self, w, mask, gen):
        if not hasattr(self, "goal"):
            self.goal = torch.zeros(w.E, dtype=torch.long, device=w.device)
            self.lcol = torch.tensor(self.LCOL, dtype=w.dtype, device=w.device)[: w.t.nL]
        self.goal = torch.where(mask, _choice(gen, w.E, w.t.nL, w.device), self.goal)
        self._place(w, mask, gen, 1.0, 1.0)

    def observation(self, w):
        speaker = self.lcol[self.goal]
        ap, lp = w.apos, w.lpos
        listener = torch.cat([w.vel[:, 1], (lp - ap[:, 1:2]).flatten(1), w.c[:, 0]], 1)
        return [speaker, listener]

    def reward(self, w):
        gl = _gather_rows(w.lpos, self.goal)
        r = -((w.apos[:, 1] - gl) ** 2).sum(1)
        return torch.stack([r, r], 1)


class SimplePush(Scenario):
    name, dim_c = "simple_push", 2

    def make(self, args):
        t = EntityTable(args.num_agents, args.num_landmarks, "cpu")
        t.silent[:] = True
        t.adversary[0] = True
        t.collide[t.nA:] = False
        t.movable[t.nA:] = False
        return t

    def reset(self, w, mask, gen):
        nL = w.t.nL
        if not hasattr(self, "goal"):
            self.goal = torch.zeros(w.E, dtype=torch.long, device=w.device)
            lc = torch.full((nL, 3), 0.1, dtype=w.dtype, device=w.device)
            for i in range(nL):
                lc[i, i + 1] += 0.8
            self.lcol = lc
        self.goal = torch.where(mask, _choice(gen, w.E, nL, w.device), self.goal)
        self._place(w, mask, gen)

    def observation(self, w):
        nA, t = w.t.nA, w.t
        ap, lp = w.apos, w.lpos
        gpos = _gather_rows(lp, self.goal)
        gcol = torch.full((w.E, 3), 0.25, dtype=w.dtype, device=w.device)
        gcol = gcol + 0.5 * torch.nn.functional.one_hot(self.goal + 1, 3).to(w.dtype)
        out = []
        for i in range(nA):
            others = [j for j in range(nA) if j != i]
            rel_l = (lp - ap[:, i: i + 1]).flatten(1)
            rel_o = (ap[:, others] - ap[:, i: i + 1]).flatten(1)
            if not bool(t.adversary[i]):
                out.append(torch.cat([w.vel[:, i], gpos - ap[:, i], gcol, rel_l,
                                      self.lcol.flatten()[None].expand(w.E, -1), rel_o], 1))
            else:
                out.append(torch.cat([w.vel[:, i], rel_l, rel_o], 1))
        return out

    def reward(self, w):
        gpos = _gather_rows(w.lpos, self.goal)
        d = (w.apos - gpos[:, None]).norm(dim=-1)                       # (E, nA)
        good = ~w.t.adversary
        pos_rew = d[:, good].min(1).values
        return torch.where(w.t.adversary[None], (pos_rew[:, None] - d), -d)


class SimpleAdversary(Scenario):
    name, dim_c = "simple_adversary", 2

    def make(self, args):
        nA = args.num_agents
        t = EntityTable(nA, nA - 1, "cpu")
        t.collide[:] = False
        t.silent[:] = True
        t.adversary[0] = True
        t.size[:nA] = 0.15
        t.size[nA:] = 0.08
        t.movable[nA:] = False
        return t

    def reset(self, w, mask, gen):
        if not hasattr(self, "goal"):
            self.goal = torch.zeros(w.E, dtype=torch.long, device=w.device)
        self.goal = torch.where(mask, _choice(gen, w.E, w.t.nL, w.device), self.goal)
        self._place(w, mask, gen, 1.0, 1.0)

    def observation(self, w):
        nA, t = w.t.nA, w.t
        ap, lp = w.apos, w.lpos
        gpos = _gather_rows(lp, self.goal)
        out = []
        for i in range(nA):
            others = [j for j in range(nA) if j != i]
            rel_l = (lp - ap[:, i: i + 1]).flatten(1)
            rel_o = (ap[:, others] - ap[:, i: i + 1]).flatten(1)
            out.append(torch.cat([rel_l, rel_o], 1) if bool(t.adversary[i]) else
                       torch.cat([gpos - ap[:, i], rel_l, rel_o], 1))
        return out

    def reward(self, w):
        adv = w.t.adversary
        gpos = _gather_rows(w.lpos, self.goal)
        d = (w.apos - gpos[:, None]).norm(dim=-1)
        good_r = -d[:, ~adv].min(1).values + d[:, adv].sum(1)
        return torch.where(adv[None], -(d ** 2), good_r[:, None].expand_as(d))


class SimpleTag(Scenario):
    name, dim_c = "simple_tag", 2
    COL_R, BOUND_W = 10.0, 1.0

    def make(self, args):
        na, ng = args.num_adversaries, args.num_good_agents
        t = EntityTable(na + ng, args.num_landmarks, "cpu")
        self._agents(t, na)
        t.size[t.nA:] = 0.2
        t.movable[t.nA:] = False
        return t

    @staticmethod
    def _agents(t, na, good_size=0.05):
        nA = t.nA
        t.silent[:] = True
        t.adversary[:na] = True
        t.size[:na], t.size[na:nA] = 0.075, good_size
        t.accel[:na], t.accel[na:nA] = 3.0, 4.0
        t.max_speed[:na], t.max_speed[na:nA] = 1.0, 1.3

    def reset(self, w, mask, gen):
        self._place(w, mask, gen)

    def observation(self, w):
        nA, adv = w.t.nA, w.t.adversary
        ap, lp = w.apos, w.lpos
        out = []
        for i in range(nA):
            others = [j for j in range(nA) if j != i]
            og = [j for j in others if not bool(adv[j])]
            out.append(torch.cat([w.vel[:, i], ap[:, i], (lp - ap[:, i: i + 1]).flatten(1),
                                  (ap[:, others] - ap[:, i: i + 1]).flatten(1), w.vel[:, og].flatten(1)], 1))
        return out

    def _col_reward(self, w):
        adv = w.t.adversary
        ai = adv.nonzero().flatten().tolist()
        gi = (~adv).nonzero().flatten().tolist()
        col = w.collisions(gi, ai).to(w.dtype)                          # (E, ng, na)
        r = torch.zeros(w.E, w.t.nA, dtype=w.dtype, device=w.device)
        r[:, gi] = -self.COL_R * col.sum(2)
        r[:, ai] = self.COL_R * col.sum((1, 2))[:, None]
        return r, gi, ai

    def reward(self, w):
        r, gi, ai = self._col_reward(w)
        r[:, gi] -= self.BOUND_W * _bound(w.apos[:, gi].abs()).sum(-1)
        return r


class SimpleWorldComm(SimpleTag):
    name, dim_c = "simple_world_comm", 4
    COL_R, BOUND_W = 5.0, 2.0
    N_FOOD, N_FOREST = 2, 2

    def make(self, args):
        na, ng = args.num_adversaries, args.num_good_agents
        self.n_obst = args.num_landmarks
        t = EntityTable(na + ng, self.n_obst + self.N_FOOD + self.N_FOREST, "cpu")
        self._agents(t, na, good_size=0.045)
        t.silent[:] = True
        t.silent[0] = False                       # the leader talks
        o = t.nA
        t.size[o: o + self.n_obst] = 0.2
        t.size[o + self.n_obst: o + self.n_obst + 2] = 0.03
        t.size[o + self.n_obst + 2:] = 0.3
        t.collide[o + self.n_obst:] = False
        t.movable[o:] = False
        return t

    def reset(self, w, mask, gen):
        self._place(w, mask, gen)
        E, dev, dt = w.E, w.device, w.dtype
        o = w.t.nA + self.n_obst
        extra = _u(gen, E, self.N_FOOD + self.N_FOREST, dev, dt, 0.8)
        p = w.pos.clone()
        p[:, o:] = extra
        w.pos = torch.where(mask[:, None, None], p, w.pos)

    def _idx(self, w):
        o = w.t.nA + self.n_obst
        return list(range(o, o + 2)), list(range(o + 2, o + 4))

    def observation(self, w):
        nA, adv = w.t.nA, w.t.adversary
        food, forest = self._idx(w)
        ap, lp = w.apos, w.lpos
        inf = w.collisions(list(range(nA)), forest)                     # (E, nA, 2)
        sgn = lambda b: torch.where(b, 1.0, -1.0).to(w.dtype)           # noqa: E731
        out = []
        for i in range(nA):
            others = [j for j in range(nA) if j != i]
            vis = ((inf[:, i: i + 1, 0] & inf[:, others, 0]) | (inf[:, i: i + 1, 1] & inf[:, others, 1]) |
                   (~inf[:, i: i + 1].any(-1) & ~inf[:, others].any(-1)))
            if i == 0:
                vis = torch.ones_like(vis)
            rel_o = (ap[:, others] - ap[:, i: i + 1]) * vis[..., None].to(w.dtype)
            og = [k for k, j in enumerate(others) if not bool(adv[j])]
            vel_o = w.vel[:, [others[k] for k in og]] * vis[:, og, None].to(w.dtype)
            in_forest = sgn(inf[:, i])
            base = [w.vel[:, i], ap[:, i], (lp - ap[:, i: i + 1]).flatten(1), rel_o.flatten(1)]
            if bool(adv[i]):
                out.append(torch.cat(base + [vel_o.flatten(1), in_forest, w.c[:, 0]], 1))
            else:
                out.append(torch.cat(base + [in_forest, vel_o.flatten(1)], 1))
        return out

    def reward(self, w):
        r, gi, ai = self._col_reward(w)
        food, _ = self._idx(w)
        ap = w.apos
        r[:, gi] -= self.BOUND_W * _bound(ap[:, gi].abs()).sum(-1)
        r[:, gi] += 2.0 * w.collisions(gi, food).to(w.dtype).sum(2)
        fd = (ap[:, gi, None] - w.pos[:, None, food]).norm(dim=-1).min(2).values
        r[:, gi] += 0.05 * fd
        gd = (ap[:, ai, None] - ap[:, None, gi]).norm(dim=-1).min(2).values   # (E, na)
        r[:, ai] -= 0.1 * gd
        return r


class SimpleCrypto(Scenario):
    name, dim_c = "simple_crypto", 4

    def make(self, args):
        t = EntityTable(args.num_agents, args.num_landmarks, "cpu")
        t.collide[:] = False
        t.movable[:] = False
        t.adversary[0] = True
        return t

    def reset(self, w, mask, gen):
        if not hasattr(self, "goal"):
            self.goal = torch.zeros(w.E, dtype=torch.long, device=w.device)
            self.key = torch.zeros(w.E, dtype=torch.long, device=w.device)
        self.goal = torch.where(mask, _choice(gen, w.E, w.t.nL, w.device), self.goal)
        self.key = torch.where(mask, _choice(gen, w.E, w.t.nL, w.device), self.key)
        self._place(w, mask, gen, 1.0, 1.0)

    def _onehot(self, w, idx):
        return torch.nn.functional.one_hot(idx, self.dim_c).to(w.dtype)

    def observation(self, w):
        goal, key = self._onehot(w, self.goal), self._onehot(w, self.key)
        out = []
        for i in range(w.t.nA):
            if i == 2:
                out.append(torch.cat([goal, key], 1))
            elif not bool(w.t.adversary[i]):
                out.append(torch.cat([key, w.c[:, 2]], 1))
            else:
                out.append(w.c[:, 2].clone())
        return out

    def reward(self, w):
        goal = self._onehot(w, self.goal)
        err = ((w.c - goal[:, None]) ** 2).sum(-1)                      # (E, nA)
        err = torch.where((w.c != 0).any(-1), err, torch.zeros_like(err))
        adv = w.t.adversary
        listeners = [i for i in range(w.t.nA) if not bool(adv[i]) and i != 2]
        good = -err[:, listeners].sum(1) + err[:, adv].sum(1)
        return torch.where(adv[None], -err, good[:, None].expand_as(err))


class SimpleAttack(SimpleTag):
    name = "simple_attack"

    def make(self, args):
        na, ng = args.num_adversaries, args.num_good_agents
        assert args.num_landmarks == na + ng, "should use the same number!"
        t = EntityTable(na + ng, args.num_landmarks, "cpu")
        nA = t.nA
        t.silent[:] = True
        t.adversary[:na] = True
        t.size[:nA], t.accel[:nA], t.max_speed[:nA] = 0.075, 3.0, 1.0
        t.size[nA:] = 0.2
        t.movable[nA:] = False
        self.failed = False
        return t

    def observation(self, w):
        nA = w.t.nA
        ap, lp = w.apos, w.lpos
        out = []
        for i in range(nA):
            others = [j for j in range(nA) if j != i]
            out.append(torch.cat([w.vel[:, i], ap[:, i], (lp - ap[:, i: i + 1]).flatten(1),
                                  (ap[:, others] - ap[:, i: i + 1]).flatten(1), w.vel[:, others].flatten(1)], 1))
        return out

    def reward(self, w):
        nA, adv = w.t.nA, w.t.adversary
        ap, lp = w.apos, w.lpos
        gd = (ap - lp[:, :nA]).norm(dim=-1)                             # goal i = landmark i
        r = -gd + 0.5 * (gd < w.t.size[nA: 2 * nA][None]).to(w.dtype)
        r = r - _bound(ap.abs()).sum(-1)
        ai = adv.nonzero().flatten().tolist()
        gi = (~adv).nonzero().flatten().tolist()
        d = (ap[:, gi, None] - ap[:, None, ai]).norm(dim=-1)           # (E, ng, na)
        lim = w.t.size[gi][:, None] + w.t.size[ai][None]
        r[:, gi] -= 0.1 * (d < 0.15).to(w.dtype).sum(2) + 0.5 * (d < lim).to(w.dtype).sum(2)
        r[:, ai] -= 0.5 * w.collisions(gi, ai).to(w.dtype).sum((1, 2))[:, None]
        if gi and ai:
            self.failed = True
        return r

    def info(self, w):
        return {"fail": torch.full((w.E,), bool(self.failed), device=w.device)}


SCENARIOS = {c.name: c for c in (SimpleSpread, SimpleReference, SimpleSpeakerListener, SimplePush, SimpleAdversary,
                                 SimpleTag, SimpleWorldComm, SimpleCrypto, SimpleAttack)}
SCENARIOS["simple_crypto_display"] = SimpleCrypto   # render-only variant of simple_crypto (same game)


def load(name: str, args) -> Scenario:
    name = name[:-3] if name.endswith(".py") else name
    if name not in SCENARIOS:
        raise KeyError(f"unknown MPE scenario {name!r}; available: {sorted(SCENARIOS)}")
    return SCENARIOS[name](args)
