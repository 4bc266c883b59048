"""Single-env, numpy-in / numpy-out view of the device env with the reference ``Env`` API.

Surface = ``DCML_BID_FIRST_MA_ENV_SingleProcess.Env`` (reference ``DCML_BID_FIRST_MA_ENV_SingleProcess.py:15-356``):

* ``Env(central_execution=True, fixed=False, preset=False, multi_agent=True)`` + the spaces it publishes
  (``:38-52``): ``n_agents``, ``observation_space`` (``[[7]]*A`` or ``[[7A]]`` single-agent),
  ``share_observation_space``, ``action_space`` (one Semi_Discrete space; 100 Discrete(2) + 1 continuous
  space when ``central_execution=False``; one mixed space when ``multi_agent=False``).
* ``reset(arrive_time=None, shannon_enable=False, binary=False)`` → ``obs (A,7)``, ``share (A,SOB)``,
  ``ava (A,2)`` (``:157-274``); ``multi_agent=False`` returns the flattened single-agent views.
* ``step(action, shannon_enable=False, standalone=False)`` → ``ob, s_ob, rewards (A,1), dones (A,), info,
  ava`` with ``info = [{"delay", "payment"}]`` (``:57-144``, ``DCML_Basic_Env.reorganize_step_output``).
* ``modify_preset``, ``generate_preset_data`` (``:316-353``), ``fake_reset`` (``:275-315``), ``close``.

Everything is computed by ``DeviceDCMLEnv`` (E = 1) — this class only converts layouts, so scripts written
against the reference env (e.g. the TD3 / benchmark notebooks) run unchanged on the new simulator.  Extra
keyword arguments: ``n_workers`` (the reference hard-wires 100), ``seed``, ``device``.
"""
from __future__ import annotations

import numpy as np
import torch

from .config import DCMLConfig
from .data import save_preset
from .spaces import dcml_action_spaces
from .vec_env import DeviceDCMLEnv


def _bits32(x: int):
    return [int(b) for b in f"{int(x):032b}"]


class Env:
    def __init__(self, central_execution=True, fixed=False, preset=False, multi_agent=True, master_class=None,
                 worker_class=None, n_workers=100, seed=None, device="cpu", cfg: DCMLConfig | None = None):
        self.cfg = cfg or DCMLConfig(n_workers=n_workers)
        self.central_execution = central_execution
        self.multi_agent = multi_agent
        self.fixed = fixed
        self.preset = preset
        seed = int(np.random.randint(0, 2 ** 31 - 1)) if seed is None else int(seed)
        self._seed = seed
        self._device = device
        self._envs = {}
        self._env = self._get(False)
        W = self.cfg.n_workers
        self.n_agents = W + self.cfg.extra_agents
        if multi_agent:
            self.observation_space = [[self.cfg.obs_dim]] * self.n_agents
        else:
            self.observation_space = [[self.cfg.obs_dim * self.n_agents]]
        self.share_observation_space = [[self.cfg.share_dim]]
        self.action_space = dcml_action_spaces(W, central_execution, multi_agent, self.cfg.action_dim,
                                               self.cfg.extra_agents)
        self.disable_rate = 50
        self._binary = False
        self._last = None

    # the Shannon flag changes the share layout, so each setting keeps its own device env (same seed)
    def _get(self, shannon: bool) -> DeviceDCMLEnv:
        if shannon not in self._envs:
            import dataclasses
            cfg = dataclasses.replace(self.cfg, shannon=bool(shannon))
            self._envs[shannon] = DeviceDCMLEnv(1, cfg, device=self._device, seed=self._seed, fixed=self.fixed,
                                                preset=self.preset)
        return self._envs[shannon]

    @property
    def eval_episode_i(self):
        return int(self._env.preset_idx[0])

    # ------------------------------------------------------------------------------------------ API
    def reset(self, arrive_time=None, shannon_enable=False, binary=False):
        self._env = self._get(bool(shannon_enable))
        self._binary = binary
        if self._last is None or self._env is not self._last:
            self._env.reset()
            self._last = self._env
        else:
            self._env._reset(torch.ones(1, dtype=torch.bool, device=self._env.device))
        if arrive_time is not None:
            self._env.arrive.fill_(int(arrive_time) % self.cfg.period)
            self._env._build_obs()
        self.arrive_time = int(self._env.arrive[0])
        self.disable_rate = int(self._env.n_disable[0])
        return self._views(self._env.obs, self._env.share)

    def _views(self, obs_t, share_t):
        obs = obs_t[0].detach().cpu().numpy().astype(np.float64)
        share = share_t[0].detach().cpu().numpy().astype(np.float64)
        if self._binary:   # R, C as 32-bit binary strings (:162-172); obs carries the first two share entries
            e = self._env
            bits = _bits32(int(e.R[0])) + _bits32(int(e.C[0]))
            share = np.concatenate([np.array(bits, dtype=np.float64), share[2:]])
            obs[:, 0], obs[:, 1] = bits[0], bits[1]
        ava = self._env.ava[0].detach().cpu().numpy().astype(np.int64)
        if self.multi_agent:
            return obs, np.tile(share, (self.n_agents, 1)), ava
        return obs.reshape(-1), share.reshape(-1), ava

    def step(self, action, shannon_enable=False, standalone=False):
        e = self._env
        a = torch.as_tensor(np.asarray(action, dtype=np.float32).reshape(1, -1), device=e.device)
        if standalone:   # worker 0 alone with K = N = 1: the N == 0 branch (:81-92)
            a = a.clone()
            a[:, : self.cfg.n_workers] = 0
        obs, share, rew, done, delay, pay, ava = e.step(a)
        self.arrive_time = int(e.arrive[0])
        ob, s_ob, av = self._views(obs, share[:, 0])
        r, d = float(rew[0]), bool(done[0])
        info = [{"delay": float(delay[0]), "payment": float(pay[0])}]
        if self.multi_agent:
            return ob, s_ob, np.full((self.n_agents, 1), r), np.full(self.n_agents, d), info, av
        return ob, s_ob, np.array([r]), np.array([d]), info, av

    def fake_reset(self, R, C, Pr, arrive_time, shannon_enable=False, binary=True):
        """Critic-style state for a given task (``:275-315``): [R, C] (binary or normalised), Pr, then each
        worker's bid at ``arrive_time``."""
        cfg, e = self.cfg, self._env
        if binary:
            state = _bits32(R) + _bits32(C)
        else:
            state = [(R - cfg.r_min) / (cfg.r_max - cfg.r_min), (C - cfg.c_min) / (cfg.c_max - cfg.c_min)]
        state.append(0.0 if shannon_enable else Pr)
        lw = e.lw[0, :, int(arrive_time) % cfg.period].detach().cpu().numpy()
        return np.concatenate([np.asarray(state, dtype=np.float64), lw.astype(np.float64)])

    def modify_preset(self, R=None, C=None, Pr=None, disable_rate=None):
        for env in self._envs.values():
            env.modify_preset(R=R, C=C, Pr=Pr, disable_rate=disable_rate)

    def generate_preset_data(self, n_episodes, shannon_enable=False, Row=None, Col=None, Probability=None,
                             disable_rate=None, dir_name="./", seed=None):
        """Write ``master_states.npy`` (n,3: R, C, Pr) and ``worker_states.npy`` (Prs (n,W), disable (n,))
        in the reference format (``:316-343``).  Unlike the reference, a fixed ``disable_rate`` is written out
        instead of leaving the disable array empty."""
        cfg = self.cfg
        rng = np.random.default_rng(seed)
        R = rng.integers(cfg.r_min, cfg.r_hi + 1, n_episodes).astype(np.float64)
        C = rng.integers(cfg.c_min, cfg.c_hi + 1, n_episodes).astype(np.float64)
        Pr = np.zeros(n_episodes) if shannon_enable else rng.uniform(cfg.pr_min, cfg.pr_max, n_episodes)
        if Row is not None:
            R[:] = Row
        if Col is not None:
            C[:] = Col
        if Probability is not None:
            Pr[:] = Probability
        if disable_rate is None:
            dis = rng.integers(1, cfg.max_disable + 1, n_episodes)
        else:
            dis = np.full(n_episodes, int(disable_rate))
        prs = rng.uniform(cfg.pr_min, cfg.pr_max, (n_episodes, cfg.n_workers))
        save_preset(dir_name, np.stack([R, C, Pr], 1), prs, dis)
        return dir_name + "master_states.npy", dir_name + "worker_states.npy"

    def close(self):
        pass
