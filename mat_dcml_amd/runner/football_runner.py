"""MAT on Google Research Football (``mat_src/mat/runner/shared/football_runner.py``), device-resident.

Same PPO loop as ``SMACRunner`` (discrete heads, so the fused HIP decode / training kernels apply when the shapes
allow) with the football bookkeeping of the reference runner:

* per-env episode reward (mean over agents) and ``score_reward`` sums; when an episode ends both are logged as
  ``train_episode_rewards/aver_rewards`` and ``train_episode_scores/aver_scores`` (``:26-95``);
* eval: deterministic episodes until ``eval_episodes`` finished → ``eval_average_episode_rewards`` /
  ``eval_average_episode_scores`` (``:167-226``).

The env is ``SyntheticFootballEnv`` (gfootball is not installable): GRF-shaped raw observations encoded by the
reference's ``FeatureEncoder`` / ``Rewarder`` logic (batched in ``envs/football/encode.py``).
"""
from __future__ import annotations

import time

import torch

from ..envs.football.synthetic import SyntheticFootballEnv
from .smac_runner import SMACRunner


class FootballRunner(SMACRunner):
    def make_env(self, a, n_envs, seed, env_id_offset, maps=None):
        return SyntheticFootballEnv(a.scenario, a.n_agent, n_envs, device=self.device, seed=seed * 1000 + env_id_offset)

    def warmup(self):
        super().warmup()
        E = self.n_rollout_threads
        self._ep_score = torch.zeros(E, device=self.device)
        self._score_stats = torch.zeros(2, device=self.device, dtype=torch.float64)   # n, Σ score

    def _track_smac(self, reward, dones, info):
        E = reward.shape[0]
        d = dones.all(1)
        self._ep_reward += reward.reshape(E, -1).mean(1)
        self._ep_score += info["score_reward"]
        dd = d.double()
        self._done_stats += torch.stack([dd.sum(), (self._ep_reward.double() * dd).sum(), info["won"].double().sum(),
                                         info["dead_allies"].double().sum()])
        self._score_stats += torch.stack([dd.sum(), (self._ep_score.double() * dd).sum()])
        self._ep_reward *= (~d).float()
        self._ep_score *= (~d).float()

    def log(self, episode, episodes, total, start, infos):
        stats = self._done_stats.clone()
        sc = self._score_stats.clone()
        self.comm.all_reduce_sum_(stats)
        self.comm.all_reduce_sum_(sc)
        self._done_stats.zero_()
        self._score_stats.zero_()
        infos = {k: float(v) for k, v in infos.items()}
        infos["average_step_rewards"] = float(self.buffer.rewards.mean())
        if not self.comm.is_main:
            return
        fps = int(total / max(time.time() - start, 1e-9))
        a = self.all_args
        print(f"\n Scenario {a.scenario} Algo {self.algorithm_name} Exp {self.experiment_name} updates "
              f"{episode}/{episodes} episodes, total num timesteps {total}/{self.num_env_steps}, FPS {fps}.\n")
        for k, v in infos.items():
            self.writter.add_scalars(k, {k: v}, total)
        n = float(stats[0])
        if n > 0:
            r, s = float(stats[1]) / n, float(sc[1]) / n
            self.writter.add_scalars("train_episode_rewards", {"aver_rewards": r}, total)
            self.writter.add_scalars("train_episode_scores", {"aver_scores": s}, total)
            print(f"some episodes done, average rewards: {r}, scores: {s}")

    @torch.no_grad()
    def eval(self, total_num_steps=0, stride=None, n_steps=None):
        env = self.eval_envs
        obs, share, ava = env.reset()
        E = obs.shape[0]
        target = max(1, self.all_args.eval_episodes)
        ep_r = torch.zeros(E, device=self.device)
        ep_s = torch.zeros(E, device=self.device)
        rs, ss = [], []
        for _ in range(n_steps or env.spec["duration"] * ((target + E - 1) // E) + 1):
            actions = self.policy.get_actions(None, obs, ava, deterministic=True, stride=stride or 1)[1]
            obs, share, r, dones, info, ava = env.step(actions)
            ep_r += r.reshape(E, -1).mean(1)
            ep_s += info["score_reward"]
            d = dones.all(1)
            if bool(d.any()):
                rs += ep_r[d].tolist()
                ss += ep_s[d].tolist()
                ep_r, ep_s = ep_r * (~d).float(), ep_s * (~d).float()
            if len(rs) >= target:
                break
        mr = sum(rs) / len(rs) if rs else float(ep_r.mean())
        ms = sum(ss) / len(ss) if ss else float(ep_s.mean())
        if self.comm.is_main:
            self.writter.add_scalars("eval_average_episode_rewards", {"eval_average_episode_rewards": mr},
                                     total_num_steps)
            self.writter.add_scalars("eval_average_episode_scores", {"eval_average_episode_scores": ms},
                                     total_num_steps)
            print(f"eval average episode rewards: {mr}, scores: {ms}.")
        return mr, ms
