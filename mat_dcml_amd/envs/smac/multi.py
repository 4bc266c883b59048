"""Multi-map SMAC training on device: unified observation layout + task embedding, padded agents / actions.

Behaviour of the reference's multi-task SMAC (``Random_StarCraft2_Env_Multi.py`` + ``feature_translation.py``,
``train_smac_multi.py``), re-done as tensor ops over the synthetic SMAC-shaped device env:

* ``--train_maps m1 m2 …``: the E envs are split evenly over the maps (``train_smac_multi.py:18-31``), each map group
  is one ``SyntheticSMACEnv``;
* every local observation is re-encoded into the map-independent layout of ``feature_translation.py:161-280``:
  26 ally slots × 54 (5 base, shield, 10-way unified unit type at 6, last action at 16), 32 enemy slots × 16,
  4 move features, 81 own features (agent id at 54) = 2001, then the 28-dim task embedding (agent / enemy counts,
  races, unit-type mix, ``:283-292``) → 2029.  Dead agents (all-zero features) translate to zeros (``:173-174``);
  the global state is the translated local obs (``Random_StarCraft2_Env_Multi.py:462-464``);
* agents are padded to 27 and actions to 38 (``:465-478``): a padded agent's obs / state is zero with a 1 at
  position ``-(i+1)`` (the reference's fake-agent marker), all its actions are available, it is always done.

The synthetic env has no shields, so the shield column stays zero.
"""
from __future__ import annotations

import torch

from .maps import N_NO_ATTACK, get_map
from .synthetic import Discrete, SyntheticSMACEnv

TARGET_AGENTS, TARGET_ENEMIES, TARGET_ACTIONS = 27, 32, 38
ALLY_F, ENEMY_F, MOVE_F, OWN_F = 54, 16, 4, 81
LOCAL_DIM = (TARGET_AGENTS - 1) * ALLY_F + TARGET_ENEMIES * ENEMY_F + MOVE_F + OWN_F      # 2001
TASK_DIM = 28
RACE = {"T": 0, "P": 1, "Z": 2}

# map -> (agent race, enemy race, agent / enemy unit counts per unified type
#         [Marine, Medivac, Marauder, Stalker, Zealot, Colossus, Zergling, Baneling, Hydralisk, Spine Crawler])
# (smac_maps.py registry + feature_translation.py:61-112)
UNIFIED = {
    "10m_vs_11m": ("T", "T", (10, 0, 0, 0, 0, 0, 0, 0, 0, 0), (11, 0, 0, 0, 0, 0, 0, 0, 0, 0)),
    "1c3s5z": ("P", "P", (0, 0, 0, 3, 5, 1, 0, 0, 0, 0), (0, 0, 0, 3, 5, 1, 0, 0, 0, 0)),
    "25m": ("T", "T", (25, 0, 0, 0, 0, 0, 0, 0, 0, 0), (25, 0, 0, 0, 0, 0, 0, 0, 0, 0)),
    "27m_vs_30m": ("T", "T", (27, 0, 0, 0, 0, 0, 0, 0, 0, 0), (30, 0, 0, 0, 0, 0, 0, 0, 0, 0)),
    "2m_vs_1z": ("T", "P", (2, 0, 0, 0, 0, 0, 0, 0, 0, 0), (0, 0, 0, 0, 1, 0, 0, 0, 0, 0)),
    "2s3z": ("P", "P", (0, 0, 0, 2, 3, 0, 0, 0, 0, 0), (0, 0, 0, 2, 3, 0, 0, 0, 0, 0)),
    "2s_vs_1sc": ("P", "Z", (0, 0, 0, 2, 0, 0, 0, 0, 0, 0), (0, 0, 0, 0, 0, 0, 0, 0, 0, 1)),
    "3m": ("T", "T", (3, 0, 0, 0, 0, 0, 0, 0, 0, 0), (3, 0, 0, 0, 0, 0, 0, 0, 0, 0)),
    "3s5z": ("P", "P", (0, 0, 0, 3, 5, 0, 0, 0, 0, 0), (0, 0, 0, 3, 5, 0, 0, 0, 0, 0)),
    "3s5z_vs_3s6z": ("P", "P", (0, 0, 0, 3, 5, 0, 0, 0, 0, 0), (0, 0, 0, 3, 6, 0, 0, 0, 0, 0)),
    "3s_vs_3z": ("P", "P", (0, 0, 0, 3, 0, 0, 0, 0, 0, 0), (0, 0, 0, 0, 3, 0, 0, 0, 0, 0)),
    "3s_vs_4z": ("P", "P", (0, 0, 0, 3, 0, 0, 0, 0, 0, 0), (0, 0, 0, 0, 4, 0, 0, 0, 0, 0)),
    "3s_vs_5z": ("P", "P", (0, 0, 0, 3, 0, 0, 0, 0, 0, 0), (0, 0, 0, 0, 5, 0, 0, 0, 0, 0)),
    "5m_vs_6m": ("T", "T", (5, 0, 0, 0, 0, 0, 0, 0, 0, 0), (6, 0, 0, 0, 0, 0, 0, 0, 0, 0)),
    "6h_vs_8z": ("Z", "P", (0, 0, 0, 0, 0, 0, 0, 0, 6, 0), (0, 0, 0, 0, 8, 0, 0, 0, 0, 0)),
    "8m": ("T", "T", (8, 0, 0, 0, 0, 0, 0, 0, 0, 0), (8, 0, 0, 0, 0, 0, 0, 0, 0, 0)),
    "8m_vs_9m": ("T", "T", (8, 0, 0, 0, 0, 0, 0, 0, 0, 0), (9, 0, 0, 0, 0, 0, 0, 0, 0, 0)),
    "MMM": ("T", "T", (7, 1, 2, 0, 0, 0, 0, 0, 0, 0), (7, 1, 2, 0, 0, 0, 0, 0, 0, 0)),
    "MMM2": ("T", "T", (7, 1, 2, 0, 0, 0, 0, 0, 0, 0), (8, 1, 3, 0, 0, 0, 0, 0, 0, 0)),
    "bane_vs_bane": ("Z", "Z", (0, 0, 0, 0, 0, 0, 20, 4, 0, 0), (0, 0, 0, 0, 0, 0, 20, 4, 0, 0)),
    "corridor": ("P", "Z", (0, 0, 0, 0, 6, 0, 0, 0, 0, 0), (0, 0, 0, 0, 0, 0, 24, 0, 0, 0)),
    "so_many_baneling": ("P", "Z", (0, 0, 0, 0, 7, 0, 0, 0, 0, 0), (0, 0, 0, 0, 0, 0, 0, 32, 0, 0)),
}


def task_embedding(map_name: str) -> torch.Tensor:
    """``gen_task_embedding`` (feature_translation.py:283-292)."""
    s = get_map(map_name)
    ar, br, na, ne = UNIFIED[map_name]
    t = torch.zeros(TASK_DIM)
    t[0], t[1] = s.n_agents / TARGET_AGENTS, s.n_enemies / TARGET_ENEMIES
    t[2 + RACE[ar]] = 1.0
    t[5 + RACE[br]] = 1.0
    t[8:18] = torch.tensor(na, dtype=torch.float32) / TARGET_AGENTS
    t[18:28] = torch.tensor(ne, dtype=torch.float32) / TARGET_ENEMIES
    return t


def _slot_types(counts, n):
    """unified unit type of each unit slot, units of a type contiguous in the registry order"""
    out = [k for k, c in enumerate(counts) for _ in range(c)]
    return (out + [out[-1] if out else 0] * n)[:n]


class UnifiedTranslator:
    """Synthetic-env local obs (E, A, d) of one map → the unified (E, A, 2029) layout."""

    def __init__(self, map_name: str, device):
        s = get_map(map_name)
        if map_name not in UNIFIED:
            raise KeyError(f"{map_name} has no unified-layout entry (feature_translation.find_map)")
        if s.n_agents > TARGET_AGENTS or s.n_enemies > TARGET_ENEMIES:
            raise ValueError(f"{map_name} exceeds the unified layout ({TARGET_AGENTS} agents / {TARGET_ENEMIES} enemies)")
        self.spec, self.device = s, torch.device(device)
        ar, br, na, ne = UNIFIED[map_name]
        self.a_type = torch.tensor(_slot_types(na, s.n_agents), device=self.device)
        self.e_type = torch.tensor(_slot_types(ne, s.n_enemies), device=self.device)
        self.task = task_embedding(map_name).to(self.device)

    def __call__(self, obs):
        s = self.spec
        E, A, _ = obs.shape
        N, u, nA = s.n_enemies, s.unit_type_bits, s.n_actions
        o = 0
        move = obs[..., o: o + 4]
        o += 4
        ef = obs[..., o: o + N * (5 + u)].reshape(E, A, N, 5 + u)
        o += N * (5 + u)
        af = obs[..., o: o + (A - 1) * (5 + u + nA)].reshape(E, A, A - 1, 5 + u + nA)
        o += (A - 1) * (5 + u + nA)
        own = obs[..., o: o + 5 + u + nA]
        o += 5 + u + nA
        ids = obs[..., o: o + A]
        dev = obs.device
        ally = torch.zeros(E, A, TARGET_AGENTS - 1, ALLY_F, device=dev)
        valid = (af != 0).any(-1, keepdim=True).float()
        ally[:, :, : A - 1, :5] = af[..., :5]
        idx = torch.arange(A, device=dev)
        others = torch.stack([torch.cat([idx[:i], idx[i + 1:]]) for i in range(A)]) if A > 1 else idx[:0].view(1, 0)
        oth_type = self.a_type[others]                                             # (A, A-1)
        ally[:, :, : A - 1, 6:16] = torch.nn.functional.one_hot(oth_type, 10).float()[None] * valid
        ally[:, :, : A - 1, 16: 16 + nA] = af[..., 5 + u:]
        enemy = torch.zeros(E, A, TARGET_ENEMIES, ENEMY_F, device=dev)
        valid_e = (ef != 0).any(-1, keepdim=True).float()
        enemy[:, :, :N, :5] = ef[..., :5]
        enemy[:, :, :N, 6:16] = torch.nn.functional.one_hot(self.e_type, 10).float()[None, None] * valid_e
        ownf = torch.zeros(E, A, OWN_F, device=dev)
        ownf[..., :5] = own[..., :5]
        ownf[..., 6:16] = torch.nn.functional.one_hot(self.a_type, 10).float()[None]
        ownf[..., 16: 16 + nA] = own[..., 5 + u:]
        ownf[..., 54: 54 + A] = ids
        local = torch.cat([ally.flatten(2), enemy.flatten(2), move, ownf], -1)
        dead = (obs[..., : obs.shape[-1] - A] == 0).all(-1, keepdim=True)
        local = torch.where(dead, torch.zeros_like(local), local)
        return torch.cat([local, self.task.expand(E, A, TASK_DIM)], -1)


class SyntheticSMACMultiEnv:
    """E envs split over ``maps``; every output in the unified 27-agent / 2029-feature / 38-action layout."""

    def __init__(self, maps, n_envs: int, device="cpu", seed: int = 1, random_agent_order: bool = False):
        maps = list(maps)
        if n_envs % len(maps):
            raise ValueError("n_rollout_threads must be a multiple of the number of maps (train_smac_multi.py:19)")
        per = n_envs // len(maps)
        self.maps, self.E, self.device = maps, int(n_envs), torch.device(device)
        self.envs = [SyntheticSMACEnv(per, m, device=device, seed=seed + 1000 * k, random_agent_order=random_agent_order)
                     for k, m in enumerate(maps)]
        self.tr = [UnifiedTranslator(m, device) for m in maps]
        self.A, self.n_actions = TARGET_AGENTS, TARGET_ACTIONS
        self.limit = max(e.spec.limit for e in self.envs)
        self.spec = type("MultiSpec", (), {"limit": self.limit})()

    @property
    def n_agents(self):
        return self.A

    @property
    def observation_space(self):
        return [[LOCAL_DIM + TASK_DIM]] * self.A

    @property
    def share_observation_space(self):
        return self.observation_space

    @property
    def action_space(self):
        return [Discrete(self.n_actions)] * self.A

    @property
    def battles_won(self):
        return torch.cat([e.battles_won for e in self.envs])

    @property
    def battles_game(self):
        return torch.cat([e.battles_game for e in self.envs])

    def _pad(self, k, obs, ava, dones=None):
        env = self.envs[k]
        E, A, D = obs.shape[0], self.A, LOCAL_DIM + TASK_DIM
        o = self.tr[k](obs)
        pad = A - env.A
        out = torch.zeros(E, A, D, device=self.device)
        out[:, : env.A] = o
        for i in reversed(range(pad)):   # fake agent j = env.A + (pad-1-i) carries a 1 at -(i+1)
            out[:, env.A + pad - 1 - i, D - (i + 1)] = 1.0
        av = torch.ones(E, A, self.n_actions, device=self.device)
        av[:, : env.A] = 0.0
        av[:, : env.A, : env.n_actions] = ava
        if dones is None:
            return out, av
        d = torch.ones(E, A, dtype=torch.bool, device=self.device)
        d[:, : env.A] = dones
        return out, av, d

    def reset(self):
        obs, ava = [], []
        for k, e in enumerate(self.envs):
            o, _, a = e.reset()
            o, a = self._pad(k, o, a)
            obs.append(o)
            ava.append(a)
        obs = torch.cat(obs)
        return obs, obs, torch.cat(ava)

    def step(self, actions):
        a = actions.reshape(self.E, self.A)
        per = self.E // len(self.envs)
        outs = []
        for k, e in enumerate(self.envs):
            ak = a[k * per:(k + 1) * per, : e.A].clamp(max=e.n_actions - 1)
            o, _, r, d, info, av = e.step(ak)
            o, av, d = self._pad(k, o, av, d)
            outs.append((o, r[:, :1].expand(-1, self.A, -1), d, info, av))
        obs = torch.cat([x[0] for x in outs])
        info = {key: torch.cat([x[3][key] for x in outs]) for key in outs[0][3]}
        return (obs, obs, torch.cat([x[1] for x in outs]), torch.cat([x[2] for x in outs]), info,
                torch.cat([x[4] for x in outs]))
