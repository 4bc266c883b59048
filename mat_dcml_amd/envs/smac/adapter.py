"""StarCraft II (SMAC) adapter behind the CPU process pool.

With ``--smac_backend sc2`` the SMAC runner drives real StarCraft II through ``smac`` / ``pysc2`` (the reference's
``StarCraft2_Env``, ``mat_src/mat/envs/starcraft2/StarCraft2_Env.py``) in worker processes
(``envs/vec/process_pool.py``), with the reference's per-agent obs / state / availability contract.  Neither
package nor the game is installable in this image, so constructing it raises with instructions; the synthetic
device env (``synthetic.py``) is the default backend.
"""
from __future__ import annotations


def _sc2_env_factory(map_name, seed):
    def make():
        from smac.env import StarCraft2Env  # noqa: WPS433 — external dependency, present only on SC2 hosts

        class _Wrap:
            def __init__(self):
                self.env = StarCraft2Env(map_name=map_name, seed=seed)
                info = self.env.get_env_info()
                self.n_agents = info["n_agents"]
                self.observation_space = [[info["obs_shape"]]] * self.n_agents
                self.share_observation_space = [[info["state_shape"]]] * self.n_agents
                from .synthetic import Discrete
                self.action_space = [Discrete(info["n_actions"])] * self.n_agents

            def reset(self):
                import numpy as np
                self.env.reset()
                obs = np.array(self.env.get_obs())
                state = np.tile(self.env.get_state(), (self.n_agents, 1))
                ava = np.array(self.env.get_avail_actions())
                return obs, state, ava

            def step(self, actions):
                import numpy as np
                r, done, info = self.env.step([int(a) for a in np.asarray(actions).reshape(-1)])
                obs, state, ava = np.array(self.env.get_obs()), np.tile(self.env.get_state(), (self.n_agents, 1)), \
                    np.array(self.env.get_avail_actions())
                dones = np.array([done] * self.n_agents)
                return obs, state, np.full((self.n_agents, 1), r), dones, [info] * self.n_agents, ava

            def close(self):
                self.env.close()
        return _Wrap()
    return make


def make_sc2_vec_env(args, n_envs, seed, device):
    try:
        import smac  # noqa: F401
    except ImportError as e:
        raise ImportError("--smac_backend sc2 needs the 'smac' package and a StarCraft II install "
                          "(SC2PATH); use the default synthetic backend otherwise") from e
    from ..vec.process_pool import ProcessPoolVecEnv
    fns = [_sc2_env_factory(args.map_name, seed * 1000 + i) for i in range(n_envs)]
    return ProcessPoolVecEnv(fns, device=device, n_workers=getattr(args, "n_env_workers", None))
