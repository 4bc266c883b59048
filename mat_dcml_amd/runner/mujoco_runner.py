"""MAT on multi-agent MuJoCo with faulty-node injection (``mat_src/mat/runner/shared/mujoco_runner.py``), on device.

Same PPO loop as ``SMACRunner`` (whole-sequence minibatches, continuous Gaussian heads, torch MAT path — the
fused HIP kernels cover the discrete / semi-discrete heads) with the MuJoCo episode structure of the reference:

* ``faulty_action``: the actions of agent ``--faulty_node`` are zeroed before they reach the robot, while the
  buffer keeps the policy's own actions (``:13-19, 48-51``) — a broken joint group the team must compensate;
* ``insert``: env done → masks 0, active masks stay 1 (all agents of a robot finish together, ``:134-157``);
* logging: FPS banner, ``average_step_rewards`` and the mean return of the episodes that finished
  (``:73-97``);
* eval: for every node of ``--eval_faulty_node`` run deterministic episodes with that node faulty until
  ``eval_episodes`` finished and log ``faulty_node_<n>/eval_average_episode_rewards`` / ``…_max_…``
  (``:99-103, 168-218``).

The robot is ``MujocoMultiVec`` (``envs/mujoco``): the reference's partition graphs and observation layouts
over a device-batched planar dynamics surrogate (MuJoCo itself is not installable here).
"""
from __future__ import annotations

import time

import torch

from ..envs.mujoco.multi import MujocoMultiVec
from .smac_runner import SMACRunner


def faulty_action(actions, faulty_node):
    """copy of ``actions`` (E, A, d) with agent ``faulty_node`` zeroed (no-op for a negative node)"""
    if faulty_node is None or faulty_node < 0:
        return actions
    out = actions.clone()
    out[:, faulty_node] = 0.0
    return out


def make_mujoco_env(a, n_envs, device, seed):
    return MujocoMultiVec(a.scenario, a.agent_conf, n_envs, agent_obsk=a.agent_obsk,
                          k_categories=getattr(a, "k_categories", None),
                          global_categories=getattr(a, "global_categories", None),
                          episode_limit=getattr(a, "episode_limit", 1000), device=device, seed=seed,
                          random_agent_order=getattr(a, "random_agent_order", False))


class MujocoRunner(SMACRunner):
    def make_env(self, a, n_envs, seed, env_id_offset, maps=None):
        return make_mujoco_env(a, n_envs, self.device, seed * 1000 + env_id_offset)

    def warmup(self):
        obs, share, ava = self.envs.reset()
        self.buffer.obs[0].copy_(obs)
        self.buffer.available_actions[0].copy_(ava)
        self.buffer.masks.fill_(1.0)
        self.buffer.active_masks.fill_(1.0)
        self._done_stats = torch.zeros(2, device=self.device, dtype=torch.float64)     # n episodes, Σ return

    @torch.no_grad()
    def rollout(self):
        self.trainer.prep_rollout()
        b = self.buffer
        E, A = b.E, b.A
        node = getattr(self.all_args, "faulty_node", -1)
        for step in range(self.episode_length):
            with self.timers("decode"):
                values, actions, logp = self.collect(step)
            with self.timers("env"):
                obs, share, reward, dones, info, ava = self.envs.step(faulty_action(actions, node))
            with self.timers("insert"):
                d = dones.all(1)
                self._ep_reward += reward.mean(1)[:, 0]
                self._done_stats += torch.stack([d.double().sum(), (self._ep_reward.double() * d).sum()])
                self._ep_reward *= (~d).float()
                masks = (~d).float().view(E, 1, 1).expand(E, A, 1)
                b.insert(None, obs, actions, logp, values, reward, masks, torch.ones(E, A, 1, device=obs.device),
                         ava)

    def log(self, episode, episodes, total, start, infos):
        stats = self._done_stats.clone()
        self.comm.all_reduce_sum_(stats)
        self._done_stats.zero_()
        avg = self.buffer.rewards.mean().double()
        self.comm.all_reduce_mean_(avg)
        infos = {k: float(v) for k, v in infos.items()}
        infos["average_step_rewards"] = float(avg)
        if not self.comm.is_main:
            return
        fps = int(total / max(time.time() - start, 1e-9))
        a = self.all_args
        print(f"\n Scenario {a.scenario} Algo {self.algorithm_name} Exp {self.experiment_name} updates "
              f"{episode}/{episodes} episodes, total num timesteps {total}/{self.num_env_steps}, FPS {fps}.\n")
        print(f"average_step_rewards is {infos['average_step_rewards']}.")
        for k, v in infos.items():
            self.writter.add_scalars(k, {k: v}, total)
        if float(stats[0]) > 0:
            r = float(stats[1]) / float(stats[0])
            print(f"some episodes done, average rewards: {r}")
            self.writter.add_scalars("train_episode_rewards", {"aver_rewards": r}, total)

    @torch.no_grad()
    def eval(self, total_num_steps=0, stride=None, n_steps=None):
        nodes = getattr(self.all_args, "eval_faulty_node", None) or [-1]
        return {node: self.eval_node(total_num_steps, node, n_steps) for node in nodes}

    @torch.no_grad()
    def eval_node(self, total_num_steps, faulty_node, n_steps=None):
        env = self.eval_envs
        obs, share, ava = env.reset()
        E = obs.shape[0]
        target = max(1, self.all_args.eval_episodes)
        ep_r = torch.zeros(E, device=self.device)
        done_r = []
        limit = n_steps or env.episode_limit * ((target + E - 1) // E) + 1
        for _ in range(limit):
            actions = self.policy.get_actions(None, obs, ava, deterministic=True)[1]
            obs, share, r, dones, info, ava = env.step(faulty_action(actions, faulty_node))
            ep_r += r.mean(1)[:, 0]
            d = dones.all(1)
            if bool(d.any()):
                done_r += ep_r[d].tolist()
                ep_r = ep_r * (~d).float()
            if len(done_r) >= target:
                break
        if not done_r:                      # n_steps cut the episodes short: report the partial returns
            done_r = ep_r.tolist()
        mean, best = sum(done_r) / len(done_r), max(done_r)
        if self.comm.is_main:
            key = f"faulty_node_{faulty_node}"
            self.writter.add_scalars(f"{key}/eval_average_episode_rewards",
                                     {f"{key}/eval_average_episode_rewards": mean}, total_num_steps)
            self.writter.add_scalars(f"{key}/eval_max_episode_rewards", {f"{key}/eval_max_episode_rewards": best},
                                     total_num_steps)
            print(f"faulty_node {faulty_node} eval_average_episode_rewards is {mean}.")
        return mean, best
