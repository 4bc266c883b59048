"""Batched Google Research Football observation / reward encoders (all envs × controlled players at once).

Reference: ``mat_src/mat/envs/football/encode/obs_encode.py`` (``FeatureEncoder.encode`` ``:20-140``,
``_get_avail_new`` ``:221-316``, ``_encode_ball_which_zone`` ``:318-342``, ``_encode_role_onehot`` ``:344-347``) and
``encode/rew_encode.py`` (``Rewarder.calc_reward`` ``:9-22`` and its terms ``:25-105``), which work on ONE raw GRF
observation dict per call.  Here a raw observation is a dict of tensors with a leading env axis E — ``left_team``
(E, NL, 2), ``left_team_direction`` (E, NL, 2), ``left_team_roles`` (E, NL), ``left_team_tired_factor`` /
``left_team_yellow_card`` (E, NL), the same for ``right_team*`` with NR, ``ball`` / ``ball_direction`` (E, 3),
``ball_owned_team`` / ``ball_owned_player`` / ``game_mode`` / ``steps_left`` (E,), ``score`` (E, 2) — plus the
per-controlled-player ``active`` (E, A) and ``sticky_actions`` (E, A, 10).  ``encode`` returns the reference's
``np.hstack`` of the feature dict in sorted-key order (``football_env.py:37-43``), i.e.
[avail (19) | ball (18) | left_closest (7) | left_team ((NL-1)·7) | player (19) | right_closest (7) |
right_team (NR·7)], as one (E, A, D) tensor, and the (E, A, 19) availability mask.
"""
from __future__ import annotations

import torch

N_ACTIONS = 19
(NO_OP, LEFT, TOP_LEFT, TOP, TOP_RIGHT, RIGHT, BOTTOM_RIGHT, BOTTOM, BOTTOM_LEFT, LONG_PASS, HIGH_PASS, SHORT_PASS,
 SHOT, SPRINT, RELEASE_MOVE, RELEASE_SPRINT, SLIDE, DRIBBLE, RELEASE_DRIBBLE) = range(19)
MIDDLE_X, PENALTY_X, END_X = 0.2, 0.64, 1.0
PENALTY_Y, END_Y = 0.27, 0.42


def ball_zone(bx, by):
    """index of the first matching zone of ``_encode_ball_which_zone`` (0..5), and the zone reward."""
    z = torch.full_like(bx, 5, dtype=torch.long)
    conds = [
        (-END_X <= bx) & (bx < -PENALTY_X) & (-PENALTY_Y < by) & (by < PENALTY_Y),
        (-END_X <= bx) & (bx < -MIDDLE_X) & (-END_Y < by) & (by < END_Y),
        (-MIDDLE_X <= bx) & (bx <= MIDDLE_X) & (-END_Y < by) & (by < END_Y),
        (PENALTY_X < bx) & (bx <= END_X) & (-PENALTY_Y < by) & (by < PENALTY_Y),
        (MIDDLE_X < bx) & (bx <= END_X) & (-END_Y < by) & (by < END_Y),
    ]
    for i in reversed(range(5)):          # first matching condition wins
        z = torch.where(conds[i], torch.full_like(z, i), z)
    return z


_ZONE_REWARD = torch.tensor([-2.0, -1.0, 0.0, 2.0, 1.0, 0.0])


def _avail(obs, ball_dist, sticky):
    """``_get_avail_new`` for (E, A)"""
    E, A = ball_dist.shape
    dev = ball_dist.device
    av = torch.ones(E, A, N_ACTIONS, device=dev)
    own = obs["ball_owned_team"].view(E, 1).expand(E, A)
    gm = obs["game_mode"].view(E, 1).expand(E, A)
    far = ball_dist > 0.03
    opp = own == 1
    free_far = (own == -1) & far & (gm == 0)
    mine = ~opp & ~free_far
    kick = [LONG_PASS, HIGH_PASS, SHORT_PASS, SHOT, DRIBBLE]

    def zero(mask, idx):
        av[..., idx] = torch.where(mask[..., None], torch.zeros_like(av[..., idx]), av[..., idx])

    zero(opp, kick)
    zero(opp & far, [SLIDE])
    zero(free_far, kick + [SLIDE])
    zero(mine, [SLIDE])
    zero(mine & far, kick)
    zero(sticky[..., 8] == 0, [RELEASE_SPRINT])
    zero(sticky[..., 9] == 1, [SLIDE])
    zero(sticky[..., 9] != 1, [RELEASE_DRIBBLE])
    zero(sticky[..., :8].sum(-1) == 0, [RELEASE_MOVE])
    bx = obs["ball"][:, 0].view(E, 1).expand(E, A)
    by = obs["ball"][:, 1].view(E, 1).expand(E, A)
    no_shot = (bx < 0.64) | (by < -0.27) | (0.27 < by)
    zero(no_shot, [SHOT])
    zero(~no_shot & (0.64 <= bx) & (bx <= 1.0) & (-0.27 <= by) & (by <= 0.27), [HIGH_PASS, LONG_PASS])
    set_piece = torch.zeros(N_ACTIONS, device=dev)
    gk = (gm == 2) & (bx < -0.7)
    ck = ~gk & (gm == 4) & (bx > 0.9)
    pk = ~gk & ~ck & (gm == 6) & (bx > 0.6)
    passes = set_piece.clone()
    passes[[NO_OP, LONG_PASS, HIGH_PASS, SHORT_PASS]] = 1.0
    shot = set_piece.clone()
    shot[[NO_OP, SHOT]] = 1.0
    av = torch.where((gk | ck)[..., None], passes.expand_as(av), av)
    av = torch.where(pk[..., None], shot.expand_as(av), av)
    return av


def encode(obs):
    """-> (features (E, A, D) float32, avail (E, A, 19))"""
    act = obs["active"].long()                                              # (E, A)
    E, A = act.shape
    lt, ld = obs["left_team"].float(), obs["left_team_direction"].float()
    NL = lt.shape[1]
    g2 = lambda t, idx: t.gather(1, idx[..., None].expand(-1, -1, t.shape[-1]))
    ppos = g2(lt, act)                                                       # (E, A, 2)
    pdir = g2(ld, act)
    pspeed = pdir.norm(dim=-1, keepdim=True)
    role = obs["left_team_roles"].long().gather(1, act)
    role_oh = torch.nn.functional.one_hot(role, 10).float()
    tired_all = obs["left_team_tired_factor"].float()
    ptired = tired_all.gather(1, act)[..., None]
    sticky = obs["sticky_actions"].float()
    ball = obs["ball"].float()                                               # (E, 3)
    bdir = obs["ball_direction"].float()
    brel = ball[:, None, :2] - ppos                                          # (E, A, 2)
    bdist = brel.norm(dim=-1)
    bspeed = bdir[:, :2].norm(dim=-1)
    own = obs["ball_owned_team"].view(E)
    owned = (own != -1).float()
    ours = (own == 0).float()
    zone = torch.nn.functional.one_hot(ball_zone(ball[:, 0], ball[:, 1]), 6).float()
    avail = _avail(obs, bdist, sticky)
    far = (bdist > 0.03).float()[..., None]
    player = torch.cat([ppos, pdir * 100, pspeed * 100, role_oh, far, ptired, sticky[..., 9:10], sticky[..., 8:9]],
                       -1)
    ball_state = torch.cat([ball[:, None].expand(E, A, 3), zone[:, None].expand(E, A, 6), brel,
                            (bdir * 20)[:, None].expand(E, A, 3), (bspeed * 20)[:, None, None].expand(E, A, 1),
                            bdist[..., None], owned.view(E, 1, 1).expand(E, A, 1), ours.view(E, 1, 1).expand(E, A, 1)],
                           -1)
    # teammates without the active player (np.delete) — (E, A, NL-1)
    ar = torch.arange(NL, device=act.device)
    others = ar[None, None, :].expand(E, A, NL)
    keep = others != act[..., None]
    oidx = others[keep].view(E, A, NL - 1)
    gath = lambda t: t[:, None].expand(E, A, *t.shape[1:]).gather(2, oidx[..., None].expand(-1, -1, -1, t.shape[-1]))
    olt, old = gath(lt), gath(ld)
    otired = tired_all[:, None].expand(E, A, NL).gather(2, oidx)[..., None]
    ldist = (olt - ppos[:, :, None]).norm(dim=-1, keepdim=True)
    lstate = torch.cat([olt * 2, old * 100, old.norm(dim=-1, keepdim=True) * 100, ldist * 2, otired], -1)
    lclose = lstate.gather(2, ldist.argmin(2, keepdim=True).expand(-1, -1, 1, 7))[:, :, 0]
    rt, rd = obs["right_team"].float(), obs["right_team_direction"].float()
    NR = rt.shape[1]
    rdist = (rt[:, None] - ppos[:, :, None]).norm(dim=-1, keepdim=True)     # (E, A, NR, 1)
    rtired = obs["right_team_tired_factor"].float()[:, None, :, None].expand(E, A, NR, 1)
    rstate = torch.cat([(rt * 2)[:, None].expand(E, A, NR, 2), (rd * 100)[:, None].expand(E, A, NR, 2),
                        (rd.norm(dim=-1, keepdim=True) * 100)[:, None].expand(E, A, NR, 1), rdist * 2, rtired], -1)
    rclose = rstate.gather(2, rdist.argmin(2, keepdim=True).expand(-1, -1, 1, 7))[:, :, 0]
    feats = torch.cat([avail, ball_state, lclose, lstate.reshape(E, A, -1), player, rclose, rstate.reshape(E, A, -1)],
                      -1)
    return feats, avail


def reward(rew, prev_obs, obs):
    """``Rewarder.calc_reward`` for every (env, controlled player): rew (E, A) scoring signal -> (E, A)"""
    E, A = rew.shape
    steps_left = obs["steps_left"].view(E)
    sc = obs["score"].float()
    win = torch.where((steps_left == 0) & (sc[:, 0] > sc[:, 1]), sc[:, 0] - sc[:, 1], torch.zeros_like(sc[:, 0]))
    ball = obs["ball"].float()
    zr = _ZONE_REWARD.to(ball.device)[ball_zone(ball[:, 0], ball[:, 1])]
    lt = obs["left_team"].float()[:, 1:]
    mind = (lt - ball[:, None, :2]).norm(dim=-1).min(1).values
    mind = torch.where(obs["ball_owned_team"].view(E) != 0, mind, torch.zeros_like(mind))
    yel = lambda o, side: o[f"{side}_team_yellow_card"].float().sum(1)
    yellow = (yel(obs, "right") - yel(prev_obs, "right")) - (yel(obs, "left") - yel(prev_obs, "left"))
    per_env = 5.0 * win + 0.003 * zr + yellow - 0.003 * mind
    return per_env[:, None] + 5.0 * rew.float()
