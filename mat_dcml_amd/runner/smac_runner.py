"""MAT on SMAC (``mat_src/mat/runner/shared/smac_runner.py``): the cross-env stress config (BASELINE #5).

Same training loop as ``DCMLRunner`` with the SMAC episode structure (``smac_runner.py:20-200``):

* ``insert``: env-level done = all agents done → masks 0 for that env; agents that died mid-episode get
  ``active_masks`` 0 (their steps are excluded from the policy / value losses), finished envs' active masks are
  reset to 1 (``:120-146``);
* logging: the incremental win rate from ``battles_won`` / ``battles_game`` deltas (``:60-80``), the dead-agent
  ratio, average step reward; eval runs deterministic episodes and reports the eval win rate (``:150-200``).

The env is the on-device ``SyntheticSMACEnv`` (StarCraft II is not available) or, with ``--smac_backend sc2`` on a
host that has it, the SC2 adapter behind the CPU process pool (``envs/smac/adapter.py``).
"""
from __future__ import annotations

import os
import time

import torch

from ..algos.buffer import RolloutBuffer
from ..algos.mat_trainer import MATTrainer
from ..algos.policy import TransformerPolicy
from ..envs.smac.synthetic import SyntheticSMACEnv
from ..parallel.comm import Comm
from ..utils.logger import ScalarWriter
from ..utils.timers import PhaseTimers
from .dcml_runner import DCMLRunner


def make_smac_env(args, n_envs, device, seed, env_id_offset=0, maps=None):
    backend = getattr(args, "smac_backend", "synthetic")
    if backend == "sc2":
        from ..envs.smac.adapter import make_sc2_vec_env
        return make_sc2_vec_env(args, n_envs, seed, device)
    rao = bool(getattr(args, "random_agent_order", False))
    if maps:   # multi-map training (train_smac_multi.py): unified layout + task embedding
        from ..envs.smac.multi import SyntheticSMACMultiEnv
        return SyntheticSMACMultiEnv(maps, n_envs, device=device, seed=seed * 1000 + env_id_offset,
                                     random_agent_order=rao)
    return SyntheticSMACEnv(n_envs, args.map_name, device=device, seed=seed * 1000 + env_id_offset,
                            random_agent_order=rao)


class SMACRunner(DCMLRunner):
    def __init__(self, config):
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
        self.train_stride, self.eval_stride = getattr(a, "train_stride", 1), 1
        E, rank = self.n_rollout_threads, self.comm.rank
        self.envs = config.get("envs") or self.make_env(a, E, a.seed, rank * E, getattr(a, "train_maps", None))
        self.eval_envs = config.get("eval_envs")
        if self.eval_envs is None and self.use_eval:
            self.eval_envs = self.make_env(a, self.n_eval_rollout_threads, a.seed + 7, rank,
                                           getattr(a, "eval_maps", None) or getattr(a, "train_maps", None))
        self.num_agents = self.envs.n_agents
        obs_dim = self.envs.observation_space[0][0]
        share_dim = self.envs.share_observation_space[0][0]
        act_space = getattr(self.envs, "policy_action_space", None) or self.envs.action_space[0]
        torch.manual_seed(a.seed)
        self.policy = TransformerPolicy(a, [obs_dim], [share_dim], act_space, self.num_agents, device=self.device)
        self.comm.broadcast_module_(self.policy.transformer)
        self.comm.seed_sampling_rng(a.seed)
        from ..ops import mat_fused   # exploration noise keyed by the global env id, as the DCML runner
        mat_fused.set_sampling_key(self.policy.transformer, a.seed, env0=rank * E)
        self.comm.attach_flat_grads(self.policy.transformer.parameters())
        self.trainer = MATTrainer(a, self.policy, self.num_agents, device=self.device, comm=self.comm)
        pol = self.policy
        self.buffer = RolloutBuffer(a.episode_length, E, self.num_agents, obs_dim, share_dim, pol.act_dim,
                                    pol.act_output_num, pol.act_prob_dim,
                                    gamma=a.gamma, gae_lambda=a.gae_lambda, use_valuenorm=a.use_valuenorm or a.use_popart,
                                    n_objective=1, device=self.device, store_share=False)
        self.log_dir = os.path.join(str(self.run_dir), "logs") if self.run_dir else None
        self.save_dir = os.path.join(str(self.run_dir), "models") if self.run_dir else None
        self.writter = ScalarWriter(self.log_dir or "/tmp/mat_dcml_logs", enabled=bool(self.run_dir) and self.comm.is_main)
        self.timers = PhaseTimers(self.device, enabled=getattr(a, "profile_phases", False))
        self.start_episode = 0
        if a.model_dir:
            self.policy.restore(a.model_dir)
            self.comm.broadcast_module_(self.policy.transformer)
        self._ep_reward = torch.zeros(E, device=self.device)
        self._done_stats = torch.zeros(4, device=self.device, dtype=torch.float64)   # n, Σreward, won, dead
        self._last_battles = torch.zeros(2, device=self.device)

    def make_env(self, a, n_envs, seed, env_id_offset, maps=None):
        return make_smac_env(a, n_envs, self.device, seed, env_id_offset, maps)

    def warmup(self):
        obs, state, ava = self.envs.reset()
        self.buffer.obs[0].copy_(obs)
        self.buffer.available_actions[0].copy_(ava)
        self.buffer.masks.fill_(1.0)
        self.buffer.active_masks.fill_(1.0)

    @torch.no_grad()
    def rollout(self):
        self.trainer.prep_rollout()
        for step in range(self.episode_length):
            with self.timers("decode"):
                values, actions, logp = self.collect(step)
            with self.timers("env"):
                obs, state, reward, dones, info, ava = self.envs.step(actions)
            with self.timers("insert"):
                if not self._insert_fused(obs, reward, dones, info, ava, values, actions, logp):
                    self._track_smac(reward, dones, info)
                    self._insert_smac(obs, reward, dones, ava, values, actions, logp)
        self._info = info

    def _insert_fused(self, obs, reward, dones, info, ava, values, actions, logp):
        """_track_smac + _insert_smac as one HIP launch (ops/kernels.smac_insert) on the device path; False -> torch."""
        b = self.buffer
        if getattr(self, "_ins_ok", None) is None:
            from ..ops import kernels
            self._ins_ok = self.device.type == "cuda" and kernels.available()
        if not self._ins_ok:
            return False
        from ..ops import kernels
        t, E, A = b.step, b.E, b.A
        pairs = [(obs, b.obs[t + 1]), (ava, b.available_actions[t + 1]), (actions, b.actions[t]),
                 (logp, b.action_log_probs[t]), (values, b.value_preds[t])]
        r = reward.reshape(E, -1)[:, 0]
        won, dead = info["won"], info["dead_allies"]
        for src, dst in pairs:
            if (src.dtype != torch.float32 or src.numel() != dst.numel() or not src.is_contiguous()
                    or not dst.is_contiguous()):
                return False
        if (dones.dtype != torch.bool or won.dtype != torch.bool or dead.dtype != torch.float32
                or b.rewards.shape[-1] != 1 or not r.is_contiguous()):
            return False
        kernels.smac_insert(pairs, r, dones.contiguous(), won.contiguous(), dead.contiguous(), b.rewards[t],
                            b.masks[t + 1], b.active_masks[t + 1], self._ep_reward, self._done_stats)
        b.step = (t + 1) % b.T
        return True

    def _track_smac(self, reward, dones, info):
        E = reward.shape[0]
        self._ep_reward += reward.reshape(E, -1)[:, 0]
        d = dones.all(1).double()
        self._done_stats += torch.stack([d.sum(), (self._ep_reward.double() * d).sum(), info["won"].double().sum(),
                                         info["dead_allies"].double().sum()])
        self._ep_reward *= (1.0 - d.float())

    def _insert_smac(self, obs, reward, dones, ava, values, actions, logp):
        b = self.buffer
        E, A = b.E, b.A
        env_done = dones.all(1, keepdim=True)                                     # (E, 1)
        masks = (~env_done).float().view(E, 1, 1).expand(E, A, 1)
        active = torch.where(env_done.view(E, 1, 1), torch.ones(E, A, 1, device=obs.device),
                             (~dones).float().view(E, A, 1))
        b.insert(None, obs, actions, logp, values, reward.reshape(E, A, 1), masks, active, ava)

    def log(self, episode, episodes, total, start, infos):
        stats = self._done_stats.clone()
        self.comm.all_reduce_sum_(stats)
        self._done_stats.zero_()
        info = getattr(self, "_info", None)
        bw = torch.stack([info["battles_won"].sum(), info["battles_game"].sum()]) if info else self._last_battles
        self.comm.all_reduce_sum_(bw)
        inc = bw - self._last_battles
        self._last_battles = bw
        incre_win_rate = float(inc[0] / inc[1]) if float(inc[1]) > 0 else 0.0
        infos = {k: float(v) for k, v in infos.items()}
        infos["average_step_rewards"] = float(self.buffer.rewards.mean())
        infos["dead_ratio"] = float(1 - self.buffer.active_masks.mean())
        if not self.comm.is_main:
            return
        fps = int(total / max(time.time() - start, 1e-9))
        print(f"\n Map {self.all_args.map_name} Algo {self.algorithm_name} Exp {self.experiment_name} updates "
              f"{episode}/{episodes} episodes, total num timesteps {total}/{self.num_env_steps}, FPS {fps}.\n")
        print(f"incre win rate is {incre_win_rate}.")
        self.writter.add_scalars("incre_win_rate", {"incre_win_rate": incre_win_rate}, total)
        for k, v in infos.items():
            self.writter.add_scalars(k, {k: v}, total)
        n = float(stats[0])
        if n > 0:
            self.writter.add_scalars("train_episode_rewards", {"aver_rewards": float(stats[1]) / n}, total)

    @torch.no_grad()
    def eval(self, total_num_steps=0, stride=None, n_steps=None):
        env = self.eval_envs
        obs, state, ava = env.reset()
        E = obs.shape[0]
        target = max(1, self.all_args.eval_episodes)
        won0, game0 = env.battles_won.sum(), env.battles_game.sum()
        ep_r = torch.zeros(E, device=self.device)
        rewards = []
        for _ in range(n_steps or (env.spec.limit * ((target + E - 1) // E) + 1)):
            actions = self.policy.get_actions(None, obs, ava, deterministic=True, stride=stride or 1)[1]
            obs, state, r, dones, info, ava = env.step(actions)
            ep_r += r[:, 0, 0]
            d = dones.all(1)
            rewards.append((ep_r * d).sum())
            ep_r *= (~d).float()
            if float(env.battles_game.sum() - game0) >= target:
                break
        games = float(env.battles_game.sum() - game0)
        win_rate = float(env.battles_won.sum() - won0) / games if games > 0 else 0.0
        avg_r = float(torch.stack(rewards).sum()) / max(games, 1.0)
        if self.comm.is_main:
            print(f"eval win rate is {win_rate}.")
            self.writter.add_scalars("eval_win_rate", {"eval_win_rate": win_rate}, total_num_steps)
            self.writter.add_scalars("eval_average_episode_rewards", {"eval_average_episode_rewards": avg_r},
                                     total_num_steps)
        return win_rate, avg_r
