"""StarCraft II (SMAC) adapter behind the CPU process pool.

With ``--smac_backend sc2`` the SMAC runner drives real StarCraft II through ``smac`` / ``pysc2`` (the reference's
``StarCraft2_Env``, ``mat_src/mat/envs/starcraft2/StarCraft2_Env.py``) in worker processes
(``envs/vec/process_pool.py``), with the reference's per-agent obs / state / availability contract.  Neither
package nor the game is installable in this image, so constructing it raises with instructions; the synthetic
device env (``synthetic.py``) is the default backend.

Protocol-error recovery (``StarCraft2_Env.py:422-423,468-472,507-530``): a ``ProtocolError`` / ``ConnectionError`` of
the SC2 client during ``reset`` or ``step`` closes the game process and launches a new one (``full_restart``); a
step that hit it ends the episode (every agent done, zero reward), and every info dict carries the running
``restarts`` count as the reference's does (``:521,603``).  The env object's episode counters (battles won / played,
timeouts) survive a restart, and the error step's info carries the reference's keys (``:517-524``).  ``SC2Game`` takes the env constructor and the error
types as arguments, so the recovery path is tested without the game (``tests/test_smac.py``).
"""
from __future__ import annotations

import numpy as np


def _protocol_errors():
    try:
        from pysc2.lib import protocol  # noqa: WPS433 — present only on SC2 hosts
        return (protocol.ProtocolError, protocol.ConnectionError)
    except ImportError:
        return (ConnectionError,)


class SC2Game:
    """One SMAC game with the reference's restart semantics.  ``make_env()`` builds a ``smac`` ``StarCraft2Env``
    (or a stand-in with its API: get_env_info / reset / step / get_obs / get_state / get_avail_actions / close)."""

    def __init__(self, make_env, errors=None, max_restarts_per_call=3):
        self.make_env = make_env
        self.errors = tuple(errors) if errors is not None else _protocol_errors()
        self.max_restarts_per_call = max_restarts_per_call
        self.force_restarts = 0
        self.env = make_env()
        info = self.env.get_env_info()
        self.n_agents = info["n_agents"]
        self.observation_space = [[info["obs_shape"]]] * self.n_agents
        self.share_observation_space = [[info["state_shape"]]] * self.n_agents
        from .synthetic import Discrete
        self.action_space = [Discrete(info["n_actions"])] * self.n_agents

    # episode counters of the env object that survive a restart: the reference relaunches only the SC2 process and
    # keeps its env object (StarCraft2_Env.py:468-472), so the runner's incremental win rate stays monotone
    _COUNTERS = ("battles_won", "battles_game", "timeouts")

    def full_restart(self):
        """Close the game process and launch a new one (StarCraft2_Env.full_restart).  smac's env relaunches its own
        process in place; an env object without that method is rebuilt with its episode counters carried over."""
        self.force_restarts += 1
        self._win_counted = bool(getattr(self.env, "win_counted", False))   # the live env's value
        if hasattr(self.env, "full_restart"):
            self.env.full_restart()
            return
        kept = {k: getattr(self.env, k) for k in self._COUNTERS if hasattr(self.env, k)}
        try:
            self.env.close()
        except Exception:   # noqa: BLE001 — the process is already gone
            pass
        self.env = self.make_env()
        for k, v in kept.items():
            setattr(self.env, k, v)

    def _error_info(self):
        """The info dict of a step that hit a protocol error (StarCraft2_Env.py:517-524)."""
        e = self.env
        # win_counted as the env object had it when the error hit (read before a rebuild replaced the object: a
        # rebuilt env starts with False); the in-place full_restart keeps the object, so its own value still holds
        won = getattr(e, "win_counted", False) if hasattr(e, "full_restart") else getattr(self, "_win_counted", False)
        return {"battles_won": getattr(e, "battles_won", 0), "battles_game": getattr(e, "battles_game", 0),
                "battles_draw": getattr(e, "timeouts", 0), "bad_transition": False, "won": bool(won)}

    def _observe(self):
        obs = np.array(self.env.get_obs())
        state = np.tile(self.env.get_state(), (self.n_agents, 1))
        ava = np.array(self.env.get_avail_actions())
        return obs, state, ava

    def reset(self):
        for attempt in range(self.max_restarts_per_call + 1):
            try:
                self.env.reset()
                return self._observe()
            except self.errors:
                if attempt == self.max_restarts_per_call:
                    raise
                self.full_restart()

    def step(self, actions):
        acts = [int(a) for a in np.asarray(actions).reshape(-1)]
        try:
            r, done, info = self.env.step(acts)
            obs, state, ava = self._observe()
        except self.errors:
            # the reference ends the episode on a protocol error after a full restart (StarCraft2_Env.py:507-530)
            self.full_restart()
            info = self._error_info()
            obs, state, ava = self.reset()
            r, done = 0.0, True
        info = dict(info or {})
        info["restarts"] = self.force_restarts
        dones = np.array([bool(done)] * self.n_agents)
        return obs, state, np.full((self.n_agents, 1), float(r)), dones, [dict(info) for _ in range(self.n_agents)], ava

    def close(self):
        self.env.close()


def _sc2_env_factory(map_name, seed):
    def make():
        def make_env():
            from smac.env import StarCraft2Env  # noqa: WPS433 — external dependency, present only on SC2 hosts
            return StarCraft2Env(map_name=map_name, seed=seed)
        return SC2Game(make_env)
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
