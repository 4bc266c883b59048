"""Vectorised MPE ``MultiAgentEnv`` on device: E worlds step together, auto-reset at ``world_length``.

Behaviour of the reference's per-world gym env (``mat_src/mat/envs/mpe/environment.py:17-280``) wrapped in its vec
env (``env_wrappers.py`` worker: reset when every agent is done), re-laid out as (E, agents, ·) tensors:

* observations: the scenario observation of agent i followed by the one-hot agent id (``environment.py:131-137``).
  Heterogeneous scenarios (speaker/listener, push, adversary, crypto, world_comm) have per-agent observation sizes;
  they are zero-padded to the largest before the id is appended, so one (E, A, obs_dim) tensor carries them all;
* actions: the reference's per-agent space is ``Discrete(5)`` (move), ``Discrete(dim_c)`` (say) or
  ``MultiDiscrete([5, dim_c])`` (both) (``environment.py:60-86``).  Here every agent takes ONE joint index
  ``a = move * n_say + say`` in ``Discrete(max_n)`` and ``available_actions`` masks the indices an agent does not
  have — so the MAT's single-categorical decoder covers every scenario (the reference MAT only handles
  ``Discrete``).  ``step_onehot`` accepts the reference runner's one-hot concatenation (``mpe_runner.py:105-115``);
* movement: one-hot ``[noop, +x, -x, +y, -y]`` → ``u = (oh1 - oh2, oh3 - oh4) · sensitivity`` (``:238-257``);
* rewards: per-agent scenario reward, replaced by the sum over agents when the world is collaborative
  (``:158-161``); ``info["individual_reward"]`` keeps the per-agent value;
* dones: ``current_step >= world_length`` for every agent (``:205-211``); finished worlds are reset and the
  returned observation is the fresh one, as the reference's vec-env worker does.
"""
from __future__ import annotations

import torch

from ..smac.synthetic import Discrete
from .core import World
from .scenarios import load


class MultiDiscrete:
    """``[[0, n0-1], [0, n1-1], …]`` (``multi_discrete.py``) — reported for reference-shaped per-agent spaces."""

    def __init__(self, bounds):
        self.low = [lo for lo, _ in bounds]
        self.high = [hi for _, hi in bounds]
        self.shape = len(bounds)
        self.n = 1
        for lo, hi in bounds:
            self.n *= hi - lo + 1


class MPEVecEnv:
    def __init__(self, args, n_envs: int, device="cpu", seed: int = 1):
        self.args = args
        self.scenario = load(args.scenario_name, args)
        self.device = torch.device(device)
        table = self.scenario.make(args)
        table.device = self.device
        self.table = table.finalize()
        self.E, self.A = int(n_envs), table.nA
        self.world = World(self.E, self.table, self.scenario.dim_c, self.device)
        self.world_length = int(self.scenario.world_length)
        self.collaborative = bool(self.scenario.collaborative)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(seed))
        heads = self.scenario.heads(self.table)
        self.n_move = torch.tensor([5 if mv else 1 for mv, _ in heads], device=self.device)
        self.n_say = torch.tensor([max(c, 1) for _, c in heads], device=self.device)
        self.has_say = torch.tensor([c > 0 for _, c in heads], device=self.device)
        self.agent_spaces = []
        for mv, c in heads:
            parts = ([[0, 4]] if mv else []) + ([[0, c - 1]] if c else [])
            self.agent_spaces.append(MultiDiscrete(parts) if len(parts) > 1 else Discrete(parts[0][1] + 1))
        n_i = self.n_move * self.n_say
        self.n_actions = int(n_i.max())
        self.ava = (torch.arange(self.n_actions, device=self.device)[None] < n_i[:, None]).float()
        self._reset_mask(torch.ones(self.E, dtype=torch.bool, device=self.device))
        raw = self.scenario.observation(self.world)
        self.raw_dims = [int(o.shape[1]) for o in raw]
        self.obs_dim = max(self.raw_dims) + self.A
        self.ep_step = torch.zeros(self.E, dtype=torch.long, device=self.device)

    # ------------------------------------------------------------------------------------- spaces
    @property
    def n_agents(self):
        return self.A

    @property
    def observation_space(self):
        return [[self.obs_dim]] * self.A

    @property
    def share_observation_space(self):
        return [[self.obs_dim * self.A]] * self.A

    @property
    def action_space(self):
        return [Discrete(self.n_actions)] * self.A

    # ------------------------------------------------------------------------------------- core
    def _reset_mask(self, mask):
        self.scenario.reset(self.world, mask, self.gen)

    def _observe(self):
        raw = self.scenario.observation(self.world)
        E, A, D = self.E, self.A, self.obs_dim - self.A
        obs = torch.zeros(E, A, self.obs_dim, device=self.device, dtype=self.world.dtype)
        for i, o in enumerate(raw):
            obs[:, i, : o.shape[1]] = o
        obs[:, :, D:] = torch.eye(A, device=self.device, dtype=obs.dtype)
        share = obs.reshape(E, 1, -1).expand(E, A, -1)
        return obs, share, self.ava[None].expand(E, -1, -1)

    def reset(self):
        self._reset_mask(torch.ones(self.E, dtype=torch.bool, device=self.device))
        self.ep_step.zero_()
        return self._observe()

    def decode_actions(self, actions):
        """joint index (E, A) -> u (E, A, 2) scaled by the sensitivity, comm one-hot (E, A, dim_c)"""
        a = actions.reshape(self.E, self.A).long()
        a = torch.minimum(a, (self.n_move * self.n_say - 1)[None])
        move, say = a // self.n_say, a % self.n_say
        u = torch.stack([(move == 1).float() - (move == 2).float(), (move == 3).float() - (move == 4).float()], -1)
        u = u * self.table.sensitivity[None, :, None]
        dc = self.world.dim_c
        comm = None
        if dc > 0:
            comm = torch.nn.functional.one_hot(say.clamp(max=dc - 1), dc).to(self.world.dtype)
            comm = comm * self.has_say[None, :, None]
        return u.to(self.world.dtype), comm

    def step_onehot(self, actions_env):
        """reference runner format: per agent the concatenated one-hots of its heads (``mpe_runner.py:105-115``)"""
        oh = actions_env.reshape(self.E, self.A, -1)
        idx = torch.zeros(self.E, self.A, dtype=torch.long, device=self.device)
        for i in range(self.A):
            nm, ns, off = int(self.n_move[i]), int(self.n_say[i]), 0
            mv = torch.zeros(self.E, dtype=torch.long, device=self.device)
            if nm > 1:
                mv = oh[:, i, :5].argmax(-1)
                off = 5
            sy = oh[:, i, off: off + ns].argmax(-1) if bool(self.has_say[i]) else torch.zeros_like(mv)
            idx[:, i] = mv * ns + sy
        return self.step(idx)

    def step(self, actions):
        """actions (E, A[, 1]) joint indices → obs, share_obs, reward (E, A, 1), dones (E, A), info, available."""
        u, comm = self.decode_actions(actions)
        self.world.step(u, comm)
        self.ep_step += 1
        r = self.scenario.reward(self.world)                                      # (E, A)
        info = {"individual_reward": r.clone()}
        info.update(self.scenario.info(self.world))
        if self.collaborative:
            r = r.sum(1, keepdim=True).expand(-1, self.A)
        done = self.ep_step >= self.world_length
        if bool(done.any()):
            self._reset_mask(done)
            self.ep_step = torch.where(done, torch.zeros_like(self.ep_step), self.ep_step)
        obs, share, ava = self._observe()
        dones = done[:, None].expand(-1, self.A)
        return obs, share, r.unsqueeze(-1), dones, info, ava
