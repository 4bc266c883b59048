"""DCML runner for the baseline algorithms (``happo``, ``rmappo``, ``ippo``, ``hatrpo``, ``ppo``, ``random``).

Reference: ``base_runner.py:64-505`` (policy / trainer / buffer construction per algorithm, ``compute``,
sequential ``train``, per-agent ``save``) driven by ``dcml_runner.py``'s loop.  In the reference only ``mat`` and
``happo`` with ``central_execution=False`` actually train on DCML; here every baseline does:

* multi-agent baselines see the DCML env with per-agent action spaces (``Env(central_execution=False)``:
  W Discrete(2) worker agents + one continuous ratio agent), per-agent actors over local obs and per-agent
  critics over the shared obs (R, C, worker loss probabilities);
* ``ppo`` is the single-agent view (``Env(multi_agent=False)``): one agent, flattened obs (7·A), one "mixed"
  action = W Categorical(2) + Normal ratio (``act.py`` MIX_ACTION);
* ``random`` uses ``algos/random_policy.py``.

Same loop, logging, checkpoint cadence and eval as ``DCMLRunner`` (device env, on-device statistics).
Checkpoints: ``models/baseline_{episode}.pt`` holding the agent-stacked actor/critic state.
"""
from __future__ import annotations

import os

import torch

from ..algos.baselines import ACPolicy, BaselineTrainer, SeparatedBuffer, _ava_dim
from ..algos.random_policy import RandomPolicy, RandomTrainer
from ..envs.dcml.config import DCMLConfig
from ..envs.dcml.spaces import dcml_action_spaces
from ..envs.dcml.vec_env import DeviceDCMLEnv
from ..parallel.comm import Comm
from ..utils.logger import ScalarWriter
from ..utils.timers import PhaseTimers
from .dcml_runner import DCMLRunner


class BaselineRunner(DCMLRunner):
    def __init__(self, config):  # noqa: C901 — mirrors the reference's per-algorithm construction
        a = config["all_args"]
        self.all_args = a
        self.comm = config.get("comm") or Comm(device=torch.device(config["device"]))
        self.device = torch.device(config["device"])
        self.run_dir = config.get("run_dir")
        self.num_env_steps, self.episode_length = a.num_env_steps, a.episode_length
        self.n_rollout_threads, self.n_eval_rollout_threads = a.n_rollout_threads, a.n_eval_rollout_threads
        self.algorithm_name, self.experiment_name = a.algorithm_name, a.experiment_name
        self.use_linear_lr_decay = a.use_linear_lr_decay
        self.save_interval, self.log_interval = a.save_interval, a.log_interval
        self.use_eval, self.eval_interval = a.use_eval, a.eval_interval
        self.train_stride, self.eval_stride = 1, 1
        self.dcml = config.get("dcml_cfg") or DCMLConfig(n_workers=a.n_workers, shannon=bool(getattr(a, "shannon", False)))
        E, rank = self.n_rollout_threads, self.comm.rank
        backend = "torch" if a.kernels == "torch" else "auto"
        self.envs = config.get("envs") or DeviceDCMLEnv(E, self.dcml, self.device, seed=a.seed, env_id_offset=rank * E,
                                                        backend=backend)
        self.eval_envs = config.get("eval_envs")
        if self.eval_envs is None and self.use_eval:
            self.eval_envs = DeviceDCMLEnv(self.n_eval_rollout_threads, self.dcml, self.device, seed=a.seed + 10007,
                                           env_id_offset=rank * self.n_eval_rollout_threads, backend=backend)
        W, A0 = self.dcml.n_workers, self.dcml.n_agents
        self.single = a.algorithm_name == "ppo"
        self.num_agents = 1 if self.single else A0
        torch.manual_seed(a.seed)
        if self.single:
            spaces = dcml_action_spaces(W, multi_agent=False)
            obs_dim = self.dcml.obs_dim * A0
        else:
            spaces = dcml_action_spaces(W, central_execution=False)
            obs_dim = self.dcml.obs_dim
        self.spaces = spaces
        if a.algorithm_name == "random":
            self.policy = RandomPolicy(a, None, None, dcml_action_spaces(W)[0], A0, self.device)
            self.trainer = RandomTrainer(a, self.policy, A0, self.device)
            self.ac = None
        else:
            if a.algorithm_name == "rmappo":
                a.use_recurrent_policy = True
            self.ac = ACPolicy(a, obs_dim, self.dcml.share_dim, spaces, self.num_agents, self.device)
            self.trainer = BaselineTrainer(a, self.ac, mode=a.algorithm_name, device=self.device)
            self.policy = self.ac
            for m in (self.ac.actors, self.ac.critic):
                self.comm.broadcast_module_(m)
        self.comm.seed_sampling_rng(a.seed)
        ava_dim = _ava_dim(("mixed", (W, 2, 1))) if self.single else 2
        act_dim = self.ac.act_dim if self.ac is not None else 1
        self.buffer = SeparatedBuffer(a, E, self.num_agents, obs_dim, self.dcml.share_dim, act_dim, ava_dim, self.device)
        self.log_dir = os.path.join(str(self.run_dir), "logs") if self.run_dir else None
        self.save_dir = os.path.join(str(self.run_dir), "models") if self.run_dir else None
        self.writter = ScalarWriter(self.log_dir or "/tmp/mat_dcml_logs", enabled=bool(self.run_dir) and self.comm.is_main)
        self.timers = PhaseTimers(self.device, enabled=getattr(a, "profile_phases", False))
        self.start_episode = 0
        if a.model_dir and self.ac is not None:
            self.ac.load_state_dict(torch.load(a.model_dir, map_location=self.device, weights_only=True))
        self._ep_reward = torch.zeros(E, device=self.device)
        self._ep_delay = torch.zeros(E, device=self.device)
        self._ep_pay = torch.zeros(E, device=self.device)
        self._done_stats = torch.zeros(4, device=self.device, dtype=torch.float64)
        self._rnn_a = self._rnn_c = None

    # ------------------------------------------------------------------------------------------ views
    def _view(self, obs, share, ava):
        """Env tensors → the agent view of this algorithm."""
        E = obs.shape[0]
        if self.single:
            W = self.dcml.n_workers
            return obs.reshape(E, 1, -1), share, ava[:, :W].reshape(E, 1, W * 2)
        return obs, share, ava

    def _env_actions(self, actions):
        E = actions.shape[0]
        return actions.reshape(E, -1)[:, : self.dcml.n_agents]

    # ------------------------------------------------------------------------------------------ rollout
    def warmup(self):
        obs, share, ava = self.envs.reset()
        o, s, av = self._view(obs, share[:, 0], ava)
        b = self.buffer
        b.obs[0].copy_(o)
        b.share_obs[0].copy_(s)
        b.available_actions[0, ..., : av.shape[-1]].copy_(av)
        b.masks.fill_(1.0)

    @torch.no_grad()
    def collect(self, step):
        b = self.buffer
        if self.ac is None:
            v, act, lp = self.policy.get_actions(None, b.obs[step], b.available_actions[step])
            return v, act, lp
        sh = b.share_obs[step][:, None].expand(b.E, b.A, -1)
        v, act, lp, ra, rc = self.ac.get_actions(sh, b.obs[step], b.rnn_states[step], b.rnn_states_critic[step],
                                                 b.masks[step], b.available_actions[step])
        self._rnn_a, self._rnn_c = ra, rc
        return v, act, lp

    @torch.no_grad()
    def rollout(self):
        self.trainer.prep_rollout()
        for step in range(self.episode_length):
            with self.timers("decode"):
                values, actions, logp = self.collect(step)
            with self.timers("env"):
                obs, share, reward, done, delay, pay, ava = self.envs.step(self._env_actions(actions))
            with self.timers("insert"):
                self._track(reward, done, delay, pay)
                self.insert(obs, share, reward, done, ava, values, actions, logp)

    def insert(self, obs, share, reward, done, ava, values, actions, logp):
        b = self.buffer
        E, A = b.E, b.A
        o, s, av = self._view(obs, share[:, 0], ava)
        masks = (~done).float().view(E, 1, 1).expand(E, A, 1)
        ra = self._rnn_a if self._rnn_a is not None else b.rnn_states[b.step]
        rc = self._rnn_c if self._rnn_c is not None else b.rnn_states_critic[b.step]
        ra = ra * masks.unsqueeze(-1)
        rc = rc * masks.unsqueeze(-1)
        acts = actions.reshape(E, A, -1)
        lp = logp.reshape(E, A, -1)
        act_full = torch.zeros_like(b.actions[0])
        lp_full = torch.zeros_like(b.action_log_probs[0])
        act_full[..., : acts.shape[-1]] = acts
        lp_full[..., : lp.shape[-1]] = lp
        b.insert(s, o, ra, rc, act_full, lp_full, values.reshape(E, A, -1)[..., :1], reward.view(E, 1, 1), masks,
                 None, av)

    def train(self):
        if self.ac is None:
            return self.trainer.train(self.buffer)
        infos = self.trainer.train(self.buffer)
        self.buffer.after_update()
        return infos

    def decide(self, obs, share, ava, stride):
        o, s, av = self._view(obs, share[:, 0], ava)
        if self.ac is None:
            return self.policy.get_actions(None, o, av, deterministic=True)[1]
        E = o.shape[0]
        rnn = torch.zeros(E, self.num_agents, self.ac.N, self.ac.H, device=o.device)
        masks = torch.ones(E, self.num_agents, 1, device=o.device)
        act = self.ac.act(s[:, None].expand(E, self.num_agents, -1), o, rnn, masks, av, deterministic=True)
        return self._env_actions(act)

    def save(self, episode):
        self.comm.barrier()
        if self.comm.is_main and self.save_dir and self.ac is not None:
            os.makedirs(self.save_dir, exist_ok=True)
            path = os.path.join(self.save_dir, f"baseline_{episode}.pt")
            tmp = path + ".tmp"
            torch.save(self.ac.state_dict(), tmp)
            os.replace(tmp, path)
