"""SMAC map parameters and the observation / state sizes they imply.

Map table: (n_agents, n_enemies, episode limit, unit-type bits) of the maps registered in the reference
(``mat_src/mat/envs/starcraft2/smac_maps.py:16-430``).  Feature sizes follow the per-entity layout of
``StarCraft2_Env.get_obs_agent`` / ``get_state_agent`` (``StarCraft2_Env.py:1559-1740``) with the reference's
default flags (``add_agent_id``, ``use_state_agent``, ``add_center_xy``, last actions in ally features):

* obs  = move 4 + enemies·(5+u) + (allies)·(5+u+n_actions) + own (5+u+n_actions) + agent id n_agents
* state = move 4 + enemies·(8+u) + (allies)·(8+u+n_actions) + own (7+u+n_actions) + agent id n_agents

For 27m_vs_30m (u = 0, 36 actions): obs 1288, state 1458.
"""
from __future__ import annotations

import dataclasses

MAPS = {
    "3m": (3, 3, 60, 0), "8m": (8, 8, 120, 0), "25m": (25, 25, 150, 0), "5m_vs_6m": (5, 6, 70, 0),
    "8m_vs_9m": (8, 9, 120, 0), "10m_vs_11m": (10, 11, 150, 0), "27m_vs_30m": (27, 30, 180, 0),
    "MMM": (10, 10, 150, 3), "MMM2": (10, 12, 180, 3), "2s3z": (5, 5, 120, 2), "3s5z": (8, 8, 150, 2),
    "3s5z_vs_3s6z": (8, 9, 170, 2), "3s_vs_3z": (3, 3, 150, 0), "3s_vs_4z": (3, 4, 200, 0),
    "3s_vs_5z": (3, 5, 250, 0), "1c3s5z": (9, 9, 180, 3), "2m_vs_1z": (2, 1, 150, 0), "corridor": (6, 24, 400, 0),
    "6h_vs_8z": (6, 8, 150, 0), "2s_vs_1sc": (2, 1, 300, 0), "so_many_baneling": (7, 32, 100, 0),
    "bane_vs_bane": (24, 24, 200, 2), "2c_vs_64zg": (2, 64, 400, 0), "1c2z_vs_1c1s1z": (3, 3, 180, 3),
    "1c2s_vs_1c1s1z": (3, 3, 180, 3), "2c1z_vs_1c1s1z": (3, 3, 180, 3), "2c1s_vs_1c1s1z": (3, 3, 180, 3),
    "1c1s1z_vs_1c1s1z": (3, 3, 180, 3), "3s5z_vs_4s4z": (8, 8, 150, 2), "4s4z_vs_4s4z": (8, 8, 150, 2),
    "5s3z_vs_4s4z": (8, 8, 150, 2), "6s2z_vs_4s4z": (8, 8, 150, 2), "2s6z_vs_4s4z": (8, 8, 150, 2),
    "6m_vs_6m_tz": (6, 6, 70, 0), "5m_vs_6m_tz": (5, 6, 70, 0), "3s6z_vs_3s6z": (9, 9, 170, 2),
    "7h_vs_8z": (7, 8, 150, 0), "2s2z_vs_zg": (4, 20, 200, 2), "1s3z_vs_zg": (4, 20, 200, 2),
    "3s1z_vs_zg": (4, 20, 200, 2), "2s2z_vs_zg_easy": (4, 18, 200, 2), "1s3z_vs_zg_easy": (4, 18, 200, 2),
    "3s1z_vs_zg_easy": (4, 18, 200, 2), "28m_vs_30m": (28, 30, 180, 0), "29m_vs_30m": (29, 30, 180, 0),
    "30m_vs_30m": (30, 30, 180, 0), "MMM2_test": (10, 12, 180, 3),
}

N_NO_ATTACK = 6   # no-op, stop, move N/S/E/W (StarCraft2_Env.py:269-271)


@dataclasses.dataclass
class SMACSpec:
    map_name: str
    n_agents: int
    n_enemies: int
    limit: int
    unit_type_bits: int

    @property
    def n_actions(self):
        return N_NO_ATTACK + self.n_enemies

    @property
    def enemy_feat(self):
        return 5 + self.unit_type_bits

    @property
    def ally_feat(self):
        return 5 + self.unit_type_bits + self.n_actions

    @property
    def own_feat(self):
        return 5 + self.unit_type_bits + self.n_actions

    @property
    def obs_dim(self):
        return 4 + self.n_enemies * self.enemy_feat + (self.n_agents - 1) * self.ally_feat + self.own_feat + self.n_agents

    @property
    def state_dim(self):
        u, n = self.unit_type_bits, self.n_actions
        return 4 + self.n_enemies * (8 + u) + (self.n_agents - 1) * (8 + u + n) + (7 + u + n) + self.n_agents

    @property
    def max_reward(self):
        """n_enemies · (max health + shield) + 10 per kill + 200 for the win (StarCraft2_Env.py:90-97); health
        is normalised to 1 per unit here, so max damage reward = n_enemies."""
        return self.n_enemies * 1.0 + self.n_enemies * 10 + 200


def get_map(name: str) -> SMACSpec:
    if name not in MAPS:
        raise KeyError(f"unknown SMAC map {name!r}; known: {sorted(MAPS)}")
    return SMACSpec(name, *MAPS[name])
