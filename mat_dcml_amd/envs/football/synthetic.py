"""Synthetic GRF-shaped football env on device (E matches at once) for the ``FootballEnv`` interface.

gfootball (and its C++ game engine) cannot be installed here, so the academy scenarios the reference trains on
(``mat_src/mat/scripts/train_football.sh``: ``academy_3_vs_1_with_keeper`` …) are re-modelled as a small 2-D
kinematic game that emits the SAME raw-observation fields GRF's ``representation="raw"`` gives the reference's
``FeatureEncoder`` (positions, directions, roles, ball, ownership, sticky actions, score, steps left).  The
observation / availability / reward encoding on top is the reference's, batched (``encode.py``); the game
mechanics are a documented surrogate:

* pitch x ∈ [-1, 1], y ∈ [-0.42, 0.42], goals at x = ±1 for |y| < 0.044; 19 GRF default actions;
* players move 0.01 / step in their sticky direction (0.015 sprinting); the owner carries the ball;
* short / high / long pass: the ball flies towards the teammate nearest to the passer's facing direction;
  shot: towards the goal mouth with noise; a free ball is taken by the nearest player within 0.015 (the keeper
  within 0.03); the defenders press the ball, the keeper tracks it on its line; an attacker being pressed loses
  the ball with probability 0.25 per step (sliding in the owner's reach steals with probability 0.5);
* academy rules: the episode ends on a goal, the ball leaving the pitch, the opponents taking possession, or
  after ``game_duration`` steps; ``score_reward`` = +1 / -1 per goal (``rewards="scoring"``).
"""
from __future__ import annotations

import torch

from . import encode as enc

# role ids (GRF e_PlayerRole): 0 GK, 1 CB, 2 LB, 3 RB, 4 DM, 5 CM, 6 LM, 7 RM, 8 AM, 9 CF
SCENARIOS = {
    # left (ours): [(x, y, role)], right: [(x, y, role)], ball owner index (left team), duration
    "academy_3_vs_1_with_keeper": dict(left=[(-1.0, 0.0, 0), (0.6, 0.0, 5), (0.7, 0.2, 6), (0.7, -0.2, 7)],
                                       right=[(1.0, 0.0, 0), (0.75, 0.0, 1)], owner=1, duration=400),
    "academy_pass_and_shoot_with_keeper": dict(left=[(-1.0, 0.0, 0), (0.7, -0.28, 5), (0.7, 0.0, 9)],
                                               right=[(1.0, 0.0, 0), (0.75, 0.1, 1)], owner=1, duration=400),
    "academy_run_pass_and_shoot_with_keeper": dict(left=[(-1.0, 0.0, 0), (0.7, -0.28, 5), (0.7, 0.0, 9)],
                                                   right=[(1.0, 0.0, 0), (0.75, 0.1, 1)], owner=2, duration=400),
    "academy_counterattack_easy": dict(left=[(-1.0, 0.0, 0), (0.2, 0.1, 5), (0.3, -0.2, 6), (0.3, 0.2, 7),
                                             (0.1, 0.0, 9)],
                                       right=[(1.0, 0.0, 0), (-0.2, 0.0, 1)], owner=1, duration=400),
    "academy_counterattack_hard": dict(left=[(-1.0, 0.0, 0), (0.2, 0.1, 5), (0.3, -0.2, 6), (0.3, 0.2, 7),
                                             (0.1, 0.0, 9)],
                                       right=[(1.0, 0.0, 0), (0.4, 0.0, 1), (0.45, 0.15, 2), (0.45, -0.15, 3)],
                                       owner=1, duration=400),
}

# idle, left, top-left, top, top-right, right, bottom-right, bottom, bottom-left (GRF's y axis points down)
_DIRS = torch.nn.functional.normalize(torch.tensor(
    [[0, 0], [-1, 0], [-1, -1], [0, -1], [1, -1], [1, 0], [1, 1], [0, 1], [-1, 1]], dtype=torch.float32), dim=-1)


class Discrete:
    def __init__(self, n):
        self.n = n
        self.shape = ()


class SyntheticFootballEnv:
    def __init__(self, scenario="academy_3_vs_1_with_keeper", n_agent=3, n_envs=1, device="cpu", seed=1):
        if scenario not in SCENARIOS:
            raise ValueError(f"unknown scenario {scenario!r}; have {sorted(SCENARIOS)}")
        self.spec = SCENARIOS[scenario]
        self.scenario = scenario
        self.device = torch.device(device)
        self.E, self.A = int(n_envs), int(n_agent)
        self.NL, self.NR = len(self.spec["left"]), len(self.spec["right"])
        if self.A > self.NL - 1:
            raise ValueError(f"{scenario} has {self.NL - 1} field players, asked to control {self.A}")
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(seed))
        f = dict(device=self.device, dtype=torch.float32)
        self.l0 = torch.tensor([p[:2] for p in self.spec["left"]], **f)
        self.r0 = torch.tensor([p[:2] for p in self.spec["right"]], **f)
        self.lroles = torch.tensor([p[2] for p in self.spec["left"]], device=self.device)
        self.dirs = _DIRS.to(self.device)
        self.active = torch.arange(1, self.A + 1, device=self.device).repeat(self.E, 1)
        self.battles_won = torch.zeros(self.E, **f)
        self.battles_game = torch.zeros(self.E, **f)
        self._reset(torch.ones(self.E, dtype=torch.bool, device=self.device))
        self.obs_dim = self.observe()[0].shape[-1]

    @property
    def n_agents(self):
        return self.A

    @property
    def observation_space(self):
        return [[self.obs_dim]] * self.A

    @property
    def share_observation_space(self):
        return [[self.obs_dim]] * self.A

    @property
    def action_space(self):
        return [Discrete(enc.N_ACTIONS)] * self.A

    # ------------------------------------------------------------------------------------ state
    def _rand(self, *shape):
        return torch.rand(*shape, generator=self.gen, device=self.device)

    def _reset(self, m):
        E = self.E
        w = lambda new, old: torch.where(m.view(-1, *([1] * (old.dim() - 1))), new, old)
        first = not hasattr(self, "lpos")
        z = lambda *s: torch.zeros(*s, device=self.device)
        if first:
            self.lpos, self.rpos = z(E, self.NL, 2), z(E, self.NR, 2)
            self.ldir, self.rdir = z(E, self.NL, 2), z(E, self.NR, 2)
            self.ball, self.bvel = z(E, 3), z(E, 3)
            self.own_team = torch.zeros(E, dtype=torch.long, device=self.device)
            self.own_player = torch.zeros(E, dtype=torch.long, device=self.device)
            self.score = z(E, 2)
            self.steps_left = torch.zeros(E, dtype=torch.long, device=self.device)
            self.sticky = z(E, self.NL, 10)
        jit = (self._rand(E, self.NL, 2) - 0.5) * 0.02
        self.lpos = w(self.l0[None] + jit * (torch.arange(self.NL, device=self.device) > 0)[None, :, None], self.lpos)
        self.rpos = w(self.r0[None].expand(E, -1, -1), self.rpos)
        self.ldir, self.rdir = w(torch.zeros_like(self.ldir), self.ldir), w(torch.zeros_like(self.rdir), self.rdir)
        o = self.spec["owner"]
        self.ball = w(torch.cat([self.lpos[:, o], torch.zeros(E, 1, device=self.device)], 1), self.ball)
        self.bvel = w(torch.zeros_like(self.bvel), self.bvel)
        self.own_team = w(torch.zeros_like(self.own_team), self.own_team)
        self.own_player = w(torch.full_like(self.own_player, o), self.own_player)
        self.score = w(torch.zeros_like(self.score), self.score)
        self.steps_left = w(torch.full_like(self.steps_left, self.spec["duration"]), self.steps_left)
        self.sticky = w(torch.zeros_like(self.sticky), self.sticky)

    def raw(self):
        E = self.E
        zl, zr = torch.zeros(E, self.NL, device=self.device), torch.zeros(E, self.NR, device=self.device)
        return {
            "left_team": self.lpos, "left_team_direction": self.ldir, "left_team_roles": self.lroles.expand(E, -1),
            "left_team_tired_factor": zl, "left_team_yellow_card": zl,
            "right_team": self.rpos, "right_team_direction": self.rdir, "right_team_tired_factor": zr,
            "right_team_yellow_card": zr, "ball": self.ball, "ball_direction": self.bvel,
            "ball_owned_team": self.own_team, "ball_owned_player": self.own_player,
            "game_mode": torch.zeros(E, dtype=torch.long, device=self.device), "score": self.score,
            "steps_left": self.steps_left, "active": self.active,
            "sticky_actions": self.sticky.gather(1, self.active[..., None].expand(-1, -1, 10)),
        }

    def observe(self):
        feats, ava = enc.encode(self.raw())
        return feats, feats, ava

    def reset(self):
        self._reset(torch.ones(self.E, dtype=torch.bool, device=self.device))
        return self.observe()

    # ------------------------------------------------------------------------------------ dynamics
    def step(self, actions):
        E, A = self.E, self.A
        dev = self.device
        prev = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in self.raw().items()}
        a = actions.reshape(E, A).long().clamp(0, enc.N_ACTIONS - 1)
        ar = torch.arange(E, device=dev)
        idx = self.active                                                    # (E, A) left-team indices
        st = self.sticky.gather(1, idx[..., None].expand(-1, -1, 10))
        # sticky directions / sprint / dribble
        mv = (a >= 1) & (a <= 8)
        st[..., :8] = torch.where(mv[..., None], torch.nn.functional.one_hot((a - 1).clamp(0, 7), 8).float(),
                                  st[..., :8])
        st[..., :8] = torch.where((a == enc.RELEASE_MOVE)[..., None], torch.zeros_like(st[..., :8]), st[..., :8])
        st[..., 8] = torch.where(a == enc.SPRINT, 1.0, torch.where(a == enc.RELEASE_SPRINT, 0.0, st[..., 8]))
        st[..., 9] = torch.where(a == enc.DRIBBLE, 1.0, torch.where(a == enc.RELEASE_DRIBBLE, 0.0, st[..., 9]))
        self.sticky = self.sticky.scatter(1, idx[..., None].expand(-1, -1, 10), st)
        dir_id = torch.where(st[..., :8].sum(-1) > 0, st[..., :8].argmax(-1) + 1, torch.zeros_like(a))
        speed = 0.01 + 0.005 * st[..., 8]
        vel = self.dirs[dir_id] * speed[..., None]                           # (E, A, 2)
        self.ldir = self.ldir.scatter(1, idx[..., None].expand(-1, -1, 2), vel)
        self.lpos = (self.lpos + self.ldir).clamp(torch.tensor([-1.0, -0.42], device=dev),
                                                  torch.tensor([1.0, 0.42], device=dev))
        # opponents: keeper tracks the ball on its line, field players press the ball
        tgt = self.ball[:, None, :2].expand(-1, self.NR, -1).clone()
        tgt[:, 0, 0] = 0.98
        tgt[:, 0, 1] = self.ball[:, 1].clamp(-0.05, 0.05)
        d = tgt - self.rpos
        self.rdir = d / d.norm(dim=-1, keepdim=True).clamp_min(1e-6) * torch.minimum(d.norm(dim=-1, keepdim=True),
                                                                                    torch.tensor(0.008, device=dev))
        self.rpos = self.rpos + self.rdir
        # ball actions of our owner
        ours = self.own_team == 0
        owner = self.own_player
        is_owner = ours[:, None] & (idx == owner[:, None])                  # (E, A)
        oa = torch.where(is_owner, a, torch.full_like(a, -1)).max(1).values  # owner's action (-1: none)
        opos = self.lpos[ar, owner]
        face = self.ldir[ar, owner]
        kick_pass = (oa == enc.SHORT_PASS) | (oa == enc.HIGH_PASS) | (oa == enc.LONG_PASS)
        shoot = oa == enc.SHOT
        # pass target: teammate (not the passer, not the keeper) best aligned with the facing direction
        rel = self.lpos - opos[:, None]
        dist = rel.norm(dim=-1).clamp_min(1e-6)
        align = (rel * face[:, None]).sum(-1) / dist / face.norm(dim=-1, keepdim=True).clamp_min(1e-6)
        score_t = -dist + 0.3 * align
        score_t[:, 0] = -1e9
        score_t[ar, owner] = -1e9
        mate = score_t.argmax(1)
        pvec = self.lpos[ar, mate] - opos
        pspeed = torch.where(oa == enc.SHORT_PASS, 0.035, 0.05)[:, None]
        pv = pvec / pvec.norm(dim=-1, keepdim=True).clamp_min(1e-6) * pspeed
        gy = (self._rand(E) - 0.5) * 0.08
        svec = torch.stack([1.0 - opos[:, 0], gy - opos[:, 1]], -1)
        sv = svec / svec.norm(dim=-1, keepdim=True).clamp_min(1e-6) * 0.07
        kicked = ours & (kick_pass | shoot)
        newv = torch.where(shoot[:, None], sv, pv)
        self.bvel = torch.where(kicked[:, None], torch.cat([newv, torch.zeros(E, 1, device=dev)], 1), self.bvel)
        self.own_team = torch.where(kicked, torch.full_like(self.own_team, -1), self.own_team)
        # carried ball follows the owner; free ball flies and slows down
        carried = self.own_team == 0
        lo = self.lpos[ar, self.own_player]
        ro = self.rpos[ar, self.own_player.clamp(max=self.NR - 1)]
        carry_pos = torch.where((self.own_team == 1)[:, None], ro, lo)
        held = self.own_team >= 0
        self.ball = torch.where(held[:, None], torch.cat([carry_pos, self.ball[:, 2:]], 1),
                                self.ball + self.bvel * (~kicked)[:, None])
        self.bvel = torch.where(held[:, None], torch.where(carried[:, None], torch.cat(
            [self.ldir[ar, self.own_player], torch.zeros(E, 1, device=dev)], 1), torch.zeros_like(self.bvel)),
            self.bvel * 0.97)
        # goals / out of play
        bx, by = self.ball[:, 0], self.ball[:, 1]
        goal_l = (bx > 1.0) & (by.abs() < 0.044)
        goal_r = (bx < -1.0) & (by.abs() < 0.044)
        out = ((bx.abs() > 1.0) | (by.abs() > 0.42)) & ~goal_l & ~goal_r
        # possession of a free ball: nearest player in reach (keeper reach 0.03)
        free = (self.own_team == -1) & ~kicked
        dl = (self.lpos - self.ball[:, None, :2]).norm(dim=-1)
        dr = (self.rpos - self.ball[:, None, :2]).norm(dim=-1)
        reach_r = torch.full((self.NR,), 0.015, device=dev)
        reach_r[0] = 0.03
        dl_min, dl_arg = dl.min(1)
        dr_ok = dr - reach_r[None]
        dr_min, dr_arg = dr_ok.min(1)
        take_l = free & (dl_min < 0.015) & ((dl_min - 0.015) <= dr_min)
        take_r = free & (dr_min < 0) & ~take_l
        # pressing: an opponent in reach of our owner steals with p = 0.25; sliding next to their owner steals
        press = (self.own_team == 0) & (dr[ar, :].min(1).values < 0.015) & (self._rand(E) < 0.25)
        slide = ((a == enc.SLIDE) & ((self.lpos.gather(1, idx[..., None].expand(-1, -1, 2)) -
                                      self.ball[:, None, :2]).norm(dim=-1) < 0.03)).any(1)
        steal = (self.own_team == 1) & slide & (self._rand(E) < 0.5)
        self.own_team = torch.where(take_l | steal, 0, torch.where(take_r | press, 1, self.own_team))
        self.own_player = torch.where(take_l, dl_arg, torch.where(take_r, dr_arg, torch.where(
            press, dr.min(1).indices, torch.where(steal, idx[:, 0], self.own_player))))
        self.bvel = torch.where((take_l | take_r | press | steal)[:, None], torch.zeros_like(self.bvel), self.bvel)
        self.score = self.score + torch.stack([goal_l.float(), goal_r.float()], 1)
        self.steps_left = self.steps_left - 1
        lost = self.own_team == 1
        done = goal_l | goal_r | out | lost | (self.steps_left <= 0)
        score_reward = goal_l.float() - goal_r.float()
        raw_now = self.raw()
        rew = enc.reward(score_reward[:, None].expand(E, A), prev, raw_now)
        self.battles_game += done.float()
        self.battles_won += (done & (self.score[:, 0] > self.score[:, 1])).float()
        info = {"score_reward": score_reward, "won": done & (self.score[:, 0] > self.score[:, 1]),
                "battles_won": self.battles_won, "battles_game": self.battles_game,
                "dead_allies": torch.zeros(E, device=dev)}
        self._reset(done)
        obs, share, ava = self.observe()
        dones = done[:, None].expand(E, A).contiguous()
        return obs, share, rew[..., None], dones, info, ava
