"""MAT on the MPE particle worlds (``mat_src/mat/runner/shared/mpe_runner.py``), device-resident.

Same PPO loop as the SMAC runner (``SMACRunner``: whole-sequence minibatches, fused HIP decode / training kernels
when the model shape allows), with the MPE episode structure of the reference runner:

* every agent is active every step; masks are 0 on the step an episode ends (``mpe_runner.py:121-137``);
* logging: ``average_episode_rewards = mean(step reward) · episode_length`` and per-agent individual rewards
  (``:60-80``); eval runs ``episode_length`` deterministic steps and reports the summed episode reward
  (``:139-189``).

The env is ``MPEVecEnv`` (all nine reference scenarios, one joint discrete action per agent with availability
masks, so the speaker / listener / comm scenarios the reference MAT cannot run train here too).
"""
from __future__ import annotations

import os
import time

import torch

from ..envs.mpe.env import MPEVecEnv
from .smac_runner import SMACRunner


class MPERunner(SMACRunner):
    def make_env(self, a, n_envs, seed, env_id_offset, maps=None):
        return MPEVecEnv(a, n_envs, device=self.device, seed=seed * 1000 + env_id_offset)

    def warmup(self):
        obs, share, ava = self.envs.reset()
        self.buffer.obs[0].copy_(obs)
        self.buffer.available_actions[0].copy_(ava)
        self.buffer.masks.fill_(1.0)
        self.buffer.active_masks.fill_(1.0)
        self._idv = torch.zeros(self.num_agents, device=self.device, dtype=torch.float64)
        self._done_stats = torch.zeros(2, device=self.device, dtype=torch.float64)     # n episodes, Σ return

    @torch.no_grad()
    def rollout(self):
        self.trainer.prep_rollout()
        b = self.buffer
        E, A = b.E, b.A
        for step in range(self.episode_length):
            with self.timers("decode"):
                values, actions, logp = self.collect(step)
            with self.timers("env"):
                obs, share, reward, dones, info, ava = self.envs.step(actions)
            with self.timers("insert"):
                self._idv += info["individual_reward"].double().sum(0)
                self._ep_reward += reward[:, 0, 0]
                d = dones[:, 0]
                self._done_stats += torch.stack([d.double().sum(), (self._ep_reward.double() * d).sum()])
                self._ep_reward *= (~d).float()
                masks = (~dones).float().view(E, A, 1)
                b.insert(None, obs, actions, logp, values, reward, masks, torch.ones(E, A, 1, device=obs.device),
                         ava)

    def log(self, episode, episodes, total, start, infos):
        stats = self._done_stats.clone()
        self.comm.all_reduce_sum_(stats)
        idv = self._idv.clone()
        self.comm.all_reduce_sum_(idv)
        n_steps = float(self.episode_length * self.n_rollout_threads * self.comm.world_size)
        self._done_stats.zero_()
        self._idv.zero_()
        avg = self.buffer.rewards.mean().double()
        self.comm.all_reduce_mean_(avg)
        infos = {k: float(v) for k, v in infos.items()}
        infos["average_episode_rewards"] = float(avg) * self.episode_length
        if not self.comm.is_main:
            return
        fps = int(total / max(time.time() - start, 1e-9))
        print(f"\n Scenario {self.all_args.scenario_name} Algo {self.algorithm_name} Exp {self.experiment_name} "
              f"updates {episode}/{episodes} episodes, total num timesteps {total}/{self.num_env_steps}, FPS {fps}.\n")
        print(f"average episode rewards is {infos['average_episode_rewards']}")
        for k, v in infos.items():
            self.writter.add_scalars(k, {k: v}, total)
        for i in range(self.num_agents):
            k = f"agent{i}/individual_rewards"
            self.writter.add_scalars(k, {k: float(idv[i]) / max(n_steps, 1.0)}, total)
        if float(stats[0]) > 0:
            self.writter.add_scalars("train_episode_rewards", {"aver_rewards": float(stats[1] / stats[0])}, total)

    @torch.no_grad()
    def eval(self, total_num_steps=0, stride=None, n_steps=None):
        env = self.eval_envs
        obs, share, ava = env.reset()
        ret = torch.zeros(env.E, device=self.device)
        for _ in range(n_steps or env.world_length):
            actions = self.policy.get_actions(None, obs, ava, deterministic=True, stride=stride or 1)[1]
            obs, share, r, dones, info, ava = env.step(actions)
            ret += r[:, 0, 0]
        avg = ret.mean().double()
        self.comm.all_reduce_mean_(avg)
        avg = float(avg)
        if self.comm.is_main:
            print("eval average episode rewards of agent: " + str(avg))
            self.writter.add_scalars("eval_average_episode_rewards", {"eval_average_episode_rewards": avg},
                                     total_num_steps)
        return avg

    @torch.no_grad()
    def render(self):
        """``render`` of the reference MPE runner (``mpe_runner.py:193-254``): ``render_episodes`` deterministic
        episodes of env 0, every frame captured when ``save_gifs`` (written to ``<run_dir>/gifs/render.gif``,
        ``ifi`` seconds per frame); prints the average episode reward.  Returns the frames."""
        from ..envs.mpe.render import render_frame, save_gif
        a = self.all_args
        env = self.envs
        frames = []
        for _ in range(a.render_episodes):
            obs, share, ava = env.reset()
            if a.save_gifs:
                frames.append(render_frame(env.world, 0))
            rewards = []
            for _ in range(self.episode_length):   # (the reference sleeps to ifi per frame for its live viewer;
                actions = self.policy.get_actions(None, obs, ava, deterministic=True)[1]   # GIF timing is ifi)
                obs, share, r, dones, info, ava = env.step(actions)
                rewards.append(r[:, 0, 0])
                if a.save_gifs:
                    frames.append(render_frame(env.world, 0))
            print("average episode rewards is: " + str(float(torch.stack(rewards).sum(0).mean())))
        if a.save_gifs and frames and self.comm.is_main:
            gif_dir = os.path.join(str(self.run_dir) if self.run_dir else ".", "gifs")
            os.makedirs(gif_dir, exist_ok=True)
            save_gif(frames, os.path.join(gif_dir, "render.gif"), a.ifi)
        return frames
