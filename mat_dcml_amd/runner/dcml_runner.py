"""DCML training / evaluation loop — one process per GPU, everything device resident.

Behavioural contract = reference ``dcml_runner.py:17-448`` + ``base_runner.py:12-505``:

* ``run`` (``dcml_runner.py:22-124``): episodes = num_env_steps // T // n_rollout_threads (per rank here);
  per episode: T rollout steps (collect → env.step → insert), compute next value + GAE, PPO train, save every
  ``save_interval`` episodes and at the last one, log every ``log_interval`` (FPS banner, average step
  reward, episode reward / delay / payment means), eval every ``eval_interval`` when ``--use_eval``.
* ``insert`` (``:250-288``): masks = 0 for envs whose agents are all done; active masks are 1 (DCML agents
  finish together).
* ``eval`` (``:319-448``): deterministic decoding with the batch decision ``stride``; reports mean episode
  reward / delay / payment and per-decision inference time.  Runs a bounded number of steps (the reference
  loops ``range(total_num_steps)``, §2.7 #7 — fixed).

MI355X design: the env is ``DeviceDCMLEnv`` (E envs as tensors, HIP env kernels), actions never leave the
GPU, episode statistics are accumulated on device and read back once per log interval, the env-id space is
partitioned by rank so the global env set does not depend on the GPU count.
"""
from __future__ import annotations

import os
import time
from contextlib import nullcontext as _null

import numpy as np
import torch

from ..algos.buffer import RolloutBuffer
from ..algos.mat_trainer import MATTrainer
from ..algos.policy import TransformerPolicy
from ..envs.dcml.config import DCMLConfig
from ..envs.dcml.spaces import dcml_action_spaces
from ..envs.dcml.vec_env import DeviceDCMLEnv
from ..parallel.comm import Comm
from ..parallel.resilience import FaultInjector, Heartbeat
from ..utils.logger import ScalarWriter
from ..utils.timers import PhaseTimers


class DCMLRunner:
    _resumed = False
    faults = FaultInjector(None)
    heartbeat = None

    def __init__(self, config):
        a = config["all_args"]
        self.all_args = a
        self.comm: Comm = config.get("comm") or Comm(device=torch.device(config["device"]))
        self.device = torch.device(config["device"])
        self.run_dir = config.get("run_dir")
        self.num_env_steps = a.num_env_steps
        self.episode_length = a.episode_length
        self.n_rollout_threads = a.n_rollout_threads
        self.n_eval_rollout_threads = a.n_eval_rollout_threads
        self.algorithm_name = a.algorithm_name
        self.experiment_name = a.experiment_name
        self.use_linear_lr_decay = a.use_linear_lr_decay
        self.save_interval, self.log_interval = a.save_interval, a.log_interval
        self.use_eval, self.eval_interval = a.use_eval, a.eval_interval
        self.train_stride, self.eval_stride = getattr(a, "train_stride", 1), getattr(a, "eval_stride", 2)
        self.dcml = config.get("dcml_cfg") or DCMLConfig(n_workers=getattr(a, "n_workers", 100),
                                                         shannon=bool(getattr(a, "shannon", False)),
                                                         alpha=float(getattr(a, "reward_alpha", 99.0)),
                                                         beta=float(getattr(a, "reward_beta", 1.0)))
        rank = self.comm.rank
        self.faults = FaultInjector(getattr(a, "fault_inject", None), rank)
        if self.faults.disable_frac is not None:
            self.dcml.disable_frac = self.faults.disable_frac
        self.heartbeat = Heartbeat(self.comm, getattr(a, "heartbeat_s", 0.0) or 0.0)
        self._resumed = False
        E = self.n_rollout_threads
        self.envs = config.get("envs") or DeviceDCMLEnv(E, self.dcml, self.device, seed=a.seed,
                                                        env_id_offset=rank * E,
                                                        backend="torch" if a.kernels == "torch" else "auto")
        self.eval_envs = config.get("eval_envs")
        if self.eval_envs is None and self.use_eval:
            self.eval_envs = DeviceDCMLEnv(self.n_eval_rollout_threads, self.dcml, self.device, seed=a.seed + 10007,
                                           env_id_offset=rank * self.n_eval_rollout_threads,
                                           backend="torch" if a.kernels == "torch" else "auto")
        self.num_agents = self.envs.n_agents
        act_space = dcml_action_spaces(self.dcml.n_workers)[0]
        torch.manual_seed(a.seed)
        self.policy = TransformerPolicy(a, self.envs.observation_space[0], self.envs.share_observation_space[0],
                                        act_space, self.num_agents, device=self.device)
        self.comm.broadcast_module_(self.policy.transformer)
        self.comm.seed_sampling_rng(a.seed)
        # exploration noise keyed by the GLOBAL env id (same key and call counter on every rank): the rollout of the
        # global env set is the same at any rank count
        from ..ops import mat_fused
        mat_fused.set_sampling_key(self.policy.transformer, a.seed, env0=rank * E)
        # every .grad is a view of ONE flat fp32 buffer: one memset to zero, one all-reduce under DP, and the fused
        # backward kernels accumulate straight into it
        self.comm.attach_flat_grads(self.policy.transformer.parameters())
        self.trainer = MATTrainer(a, self.policy, self.num_agents, device=self.device, comm=self.comm)
        self.buffer = RolloutBuffer(a.episode_length, E, self.num_agents, self.dcml.obs_dim, self.dcml.share_dim,
                                    self.dcml.action_dim, gamma=a.gamma, gae_lambda=a.gae_lambda,
                                    use_valuenorm=a.use_valuenorm or a.use_popart, n_objective=a.n_objective,
                                    use_advantage_norm=bool(getattr(a, "use_advantage_norm", False)),
                                    device=self.device)
        self.log_dir = os.path.join(str(self.run_dir), "logs") if self.run_dir else None
        self.save_dir = os.path.join(str(self.run_dir), "models") if self.run_dir else None
        self.writter = ScalarWriter(self.log_dir or "/tmp/mat_dcml_logs", enabled=bool(self.run_dir) and self.comm.is_main)
        self.timers = PhaseTimers(self.device, enabled=getattr(a, "profile_phases", False))
        self.trainer.timers = self.timers
        self.start_episode = 0
        if a.model_dir:
            self.policy.restore(a.model_dir)
            self.comm.broadcast_module_(self.policy.transformer)
        self._ep_reward = torch.zeros(E, device=self.device)
        self._ep_delay = torch.zeros(E, device=self.device)
        self._ep_pay = torch.zeros(E, device=self.device)
        self._done_stats = torch.zeros(4, device=self.device, dtype=torch.float64)  # n, Σreward, Σdelay, Σpay

    # ---------------------------------------------------------------------------------------- rollout
    def warmup(self):
        if self._resumed:   # env restored from its checkpointed counters: continue from its current task
            obs, share, ava = self.envs.obs, self.envs.share_view(), self.envs.ava
        else:
            obs, share, ava = self.envs.reset()
        self.buffer.obs[0].copy_(obs)
        self.buffer.share_obs[0].copy_(share[:, 0])
        self.buffer.available_actions[0].copy_(ava)
        self.buffer.masks.fill_(1.0)

    @torch.no_grad()
    def collect(self, step):
        b = self.buffer
        return self.policy.get_actions(None, b.obs[step], b.available_actions[step], deterministic=False,
                                       stride=self.train_stride)

    @torch.no_grad()
    def rollout(self):
        self.trainer.prep_rollout()
        G = self._groups()
        if G > 1:
            return self._rollout_groups(G)
        # the weight packs of the decode / encoder kernels are rebuilt once per optimizer step: their own phase, so
        # the first rollout step's decode does not carry them
        with self.timers("pack"):
            from ..ops import mat_fused
            mat_fused.refresh_packs(self.policy.transformer)
        for step in range(self.episode_length):
            with self.timers("decode"):
                values, actions, logp = self.collect(step)
            with self.timers("env"):
                obs, share, reward, done, delay, pay, ava = self.envs.step(actions)
            with self.timers("insert"):
                if not self._insert_fused(obs, share, reward, done, ava, values, actions, logp, delay, pay):
                    self._track(reward, done, delay, pay)
                    self.insert(obs, share, reward, done, ava, values, actions, logp, delay, pay)

    def _groups(self):
        """Env groups of the pipelined rollout (``--rollout_groups``): > 1 only where it can overlap anything (HIP
        env kernels, a CUDA device) and the rollout stays identical (globally keyed sampling noise)."""
        G = int(getattr(self.all_args, "rollout_groups", 1) or 1)
        if G <= 1 or self.n_rollout_threads % G or not hasattr(self.envs, "group_views") \
                or not hasattr(self.policy.transformer, "_mdl_env0"):
            return 1
        return G

    def _rollout_groups(self, G):
        """The rollout as G env groups, each on its own stream (SURVEY §2.4 overlap plan): group g's decode and
        group g'’s env step / insert / encoder are independent, so the device runs them side by side (the decode
        of one env per workgroup leaves most of each CU idle on its own).  Each step takes the sampling counter
        once and every group names its first global env id (``mat_fused.sampling_group``); the env groups are
        views of the one env (``group_views``), so buffers, env state and statistics equal the 1-group rollout's."""
        from ..ops import mat_fused
        b, E = self.buffer, self.n_rollout_threads
        n = E // G
        if getattr(self, "_gviews", None) is None or len(self._gviews) != G:
            self._gviews = self.envs.group_views(G)
            cuda = self.device.type == "cuda"
            self._gstreams = [torch.cuda.Stream(self.device) if cuda else None for _ in range(G)]
            self._gstats = [torch.zeros(4, device=self.device, dtype=torch.float64) for _ in range(G)]
        streams = self._gstreams
        cur = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        # every version-keyed weight pack is rebuilt HERE, on the current stream, before the groups' streams fork
        # off it: lazily on group 0's stream, group 1 would read it half-written after an optimizer step
        mat_fused.refresh_packs(self.policy.transformer)
        for s in streams:
            if s is not None:
                s.wait_stream(cur)
        sg = mat_fused.sampling_group(self.policy.transformer)
        try:
            for step in range(self.episode_length):
                sg.hold()
                for g in range(G):
                    lo, hi = g * n, (g + 1) * n
                    with torch.cuda.stream(streams[g]) if streams[g] is not None else _null():
                        sg.group(lo)
                        values, actions, logp = self.policy.get_actions(
                            None, b.obs[step][lo:hi], b.available_actions[step][lo:hi], deterministic=False,
                            stride=self.train_stride)
                        obs, share, reward, done, delay, pay, ava = self._gviews[g].step(actions)
                        self._insert_rows(lo, hi, self._gstats[g], obs, share, reward, done, ava, values, actions,
                                          logp, delay, pay)
                b.step = (b.step + 1) % b.T
        finally:
            sg.close()
            for s in streams:
                if s is not None:
                    cur.wait_stream(s)
        for st in self._gstats:   # the groups' finished-episode statistics (fixed order)
            self._done_stats += st
            st.zero_()

    def _insert_rows(self, lo, hi, stats, obs, share, reward, done, ava, values, actions, logp, delay, pay):
        """insert of env rows [lo, hi) of the current slot: the fused launch, or the torch ops on row views."""
        b, t = self.buffer, self.buffer.step
        if self._insert_fused(obs, share, reward, done, ava, values, actions, logp, delay, pay, rows=(lo, hi),
                              stats=stats, advance=False):
            return
        A = b.A
        self._ep_reward[lo:hi] += reward
        self._ep_delay[lo:hi] += delay
        self._ep_pay[lo:hi] += pay
        d = done.to(torch.float64)
        stats += torch.stack([d.sum(), (self._ep_reward[lo:hi].double() * d).sum(),
                              (self._ep_delay[lo:hi].double() * d).sum(), (self._ep_pay[lo:hi].double() * d).sum()])
        keep = (~done).float()
        self._ep_reward[lo:hi] *= keep
        self._ep_delay[lo:hi] *= keep
        self._ep_pay[lo:hi] *= keep
        m = hi - lo
        b.share_obs[t + 1][lo:hi] = share if share.dim() == 2 else share[:, 0]
        b.obs[t + 1][lo:hi] = obs
        b.available_actions[t + 1][lo:hi] = ava
        b.actions[t][lo:hi] = actions.reshape(b.actions[t][lo:hi].shape)
        b.action_log_probs[t][lo:hi] = logp.reshape(b.action_log_probs[t][lo:hi].shape)
        b.value_preds[t][lo:hi] = values.reshape(b.value_preds[t][lo:hi].shape)
        if b.n_objective == 2:
            b.rewards[t][lo:hi] = torch.stack([-delay, -pay], -1).view(m, 1, 2).expand(m, A, 2)
        else:
            b.rewards[t][lo:hi] = reward.view(m, 1, 1).expand(m, A, 1)
        b.masks[t + 1][lo:hi] = (~done).float().view(m, 1, 1).expand(m, A, 1)

    def _insert_fused(self, obs, share, reward, done, ava, values, actions, logp, delay, pay, rows=None, stats=None,
                      advance=True):
        """_track + insert as one HIP launch (ops/kernels.rollout_insert) when every operand is a contiguous f32
        device tensor of the buffer's slot size; False -> the torch path.  ``rows`` = (lo, hi): env rows of one
        rollout group (their slot rows and episode sums, statistics into ``stats``)."""
        b = self.buffer
        if getattr(self, "_ins_ok", None) is None:
            from ..ops import kernels
            self._ins_ok = (self.device.type == "cuda" and kernels.available() and b.share_obs is not None
                            and b.n_objective in (1, 2))
        if not self._ins_ok:
            return False
        from ..ops import kernels
        t = b.step
        lo, hi = rows if rows is not None else (0, b.E)
        # the buffer-side views of slot t (persistent tensors): built once per (slot, rows), not per step — the
        # rollout's host side runs only ~1.6x ahead of the GPU, and each view is a torch object to create
        key = (t, lo, hi)
        cache = self.__dict__.setdefault("_ins_views", {})
        dv = cache.get(key)
        if dv is None:
            dv = cache[key] = ([b.share_obs[t + 1][lo:hi], b.obs[t + 1][lo:hi], b.available_actions[t + 1][lo:hi],
                                b.actions[t][lo:hi], b.action_log_probs[t][lo:hi], b.value_preds[t][lo:hi]],
                               b.rewards[t][lo:hi], b.masks[t + 1][lo:hi], b.rewards[t].is_contiguous(),
                               self._ep_reward[lo:hi], self._ep_delay[lo:hi], self._ep_pay[lo:hi])
        dsts, rew_slot, mask_slot, rew_ok, ep_r, ep_d, ep_p = dv
        sh = share if share.dim() == 2 else share[:, 0]
        pairs = list(zip((sh, obs, ava, actions, logp, values), dsts))
        for src, dst in pairs:
            if (src.dtype != torch.float32 or src.numel() != dst.numel() or not src.is_contiguous()
                    or not dst.is_contiguous()):
                return False
        if done.dtype != torch.bool or not rew_ok:
            return False
        kernels.rollout_insert(pairs, reward.contiguous(), delay.contiguous(), pay.contiguous(), done.contiguous(),
                               rew_slot, mask_slot, ep_r, ep_d, ep_p, self._done_stats if stats is None else stats)
        if advance:
            b.step = (t + 1) % b.T
        return True

    def _track(self, reward, done, delay, pay):
        self._ep_reward += reward
        self._ep_delay += delay
        self._ep_pay += pay
        d = done.to(torch.float64)
        self._done_stats += torch.stack([d.sum(), (self._ep_reward.double() * d).sum(),
                                         (self._ep_delay.double() * d).sum(), (self._ep_pay.double() * d).sum()])
        keep = (~done).float()
        self._ep_reward *= keep
        self._ep_delay *= keep
        self._ep_pay *= keep

    def insert(self, obs, share, reward, done, ava, values, actions, logp, delay=None, pay=None):
        E, A = self.buffer.E, self.buffer.A
        masks = (~done).float().view(E, 1, 1).expand(E, A, 1)
        if self.buffer.n_objective == 2:   # multi-objective MAT: objectives (-completion time, -payment)
            rew = torch.stack([-delay, -pay], -1).view(E, 1, 2).expand(E, A, 2)
        else:
            rew = reward.view(E, 1, 1).expand(E, A, 1)
        self.buffer.insert(share, obs, actions, logp, values, rew, masks, None, ava)

    def compute(self):
        pass  # next-value + GAE are recomputed inside every PPO epoch (mat_trainer.py:178-192)

    def train(self):
        self.trainer.prep_training()
        infos = self.trainer.train(self.buffer)
        self.buffer.after_update()
        return infos

    def train_iteration(self):
        """One PPO iteration = T·E env steps + the update.  The unit timed by bench.py."""
        self.rollout()
        self.compute()
        with self.timers("update"):
            infos = self.train()
        return infos

    # ---------------------------------------------------------------------------------------- main loop
    def run(self):
        from ..ops.paths import log_kernel_report
        log_kernel_report(self)
        self.warmup()
        start = time.time()
        episodes = int(self.num_env_steps) // self.episode_length // self.n_rollout_threads // self.comm.world_size
        episodes = max(episodes, 1)
        last_infos = None
        for episode in range(self.start_episode, episodes):
            if self.use_linear_lr_decay:
                self.policy.lr_decay(episode, episodes)
            self.faults.maybe_kill(episode, before=self._log_flush)   # the last queued log is not lost
            self.trainer.poison = self.faults.poison_grads(episode)
            try:
                infos = self.train_iteration()
            except BaseException:
                self._log_flush()   # a faulting iteration still prints the previous interval's statistics
                raise
            total = (episode + 1) * self.episode_length * self.n_rollout_threads * self.comm.world_size
            if episode % self.save_interval == 0 or episode == episodes - 1:
                self._log_flush()
                self.save(episode)
            if episode % self.log_interval == 0:
                self.log(episode, episodes, total, start, infos)
            if self.use_eval and episode % self.eval_interval == 0:
                self._log_flush()   # this episode's log prints before the eval output (the reference's order)
                self.eval(total)
            last_infos = infos
        self._log_flush()
        return last_infos

    def log(self, episode, episodes, total, start, infos):
        """Queue this log's statistics: ONE packed asynchronous all-reduce (episode sums + per-objective average step
        reward) started here and overlapped with the next rollout; it is waited on, and the scalars are read back
        and printed, at the next ``log`` (or at the end of ``run``), so logging never drains the GPU queue or
        blocks a rank on the collective inside the training loop."""
        self._log_flush()
        packed = torch.cat([self._done_stats, self.buffer.rewards.mean((0, 1, 2)).double()])
        self._done_stats.zero_()
        work = self.comm.all_reduce_sum_async(packed)
        infos = {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in infos.items()}
        self._pending_log = (work, packed, episode, episodes, total, time.time() - start, infos)

    def _log_flush(self):
        pend = getattr(self, "_pending_log", None)
        if pend is None:
            return
        self._pending_log = None
        work, packed, episode, episodes, total, elapsed, infos = pend
        if work is not None:
            work.wait()
        stats = packed[:4]
        avg_step_reward = packed[4:] / self.comm.world_size    # per objective
        infos = {k: float(v) for k, v in infos.items()}
        infos["average_step_rewards"] = float(avg_step_reward.sum())
        if avg_step_reward.numel() > 1:   # dcml_runner.py:306-309
            for i in range(avg_step_reward.numel()):
                infos[f"average_step_objective_{i}"] = float(avg_step_reward[i])
        self.last_log = infos
        if not self.comm.is_main:
            return
        fps = int(total / max(elapsed, 1e-9))
        print(f"\n Scenario {self.all_args.scenario} Algo {self.algorithm_name} Exp {self.experiment_name} "
              f"updates {episode}/{episodes} episodes, total num timesteps {total}/{self.num_env_steps}, FPS {fps}.\n")
        print(f"average_step_rewards is {infos['average_step_rewards']}.")
        for k, v in infos.items():
            self.writter.add_scalars(k, {k: v}, total)
        n = float(stats[0])
        if n > 0:
            r, d, p = float(stats[1]) / n, float(stats[2]) / n, float(stats[3]) / n
            self.writter.add_scalars("train_episode_rewards", {"aver_rewards": r}, total)
            self.writter.add_scalars("train_episode_scores", {"aver_delay": d, "aver_payment": p}, total)
            print(f"some episodes done, average rewards: {r}, delays: {d},payments: {p}")
        if self.timers.enabled:
            print(self.timers.summary())

    def save(self, episode):
        """Checkpoint (reference layout).  No collective when nothing is written (bench / no run dir); otherwise ONE
        barrier after the writes, so a resume never sees rank 0's model without every rank's env counters."""
        if not self.save_dir:
            return
        if getattr(self.all_args, "save_trainer_state", True) and hasattr(self.envs, "task_ctr"):   # per-rank env counters
            from ..utils.checkpoint import save_env_state
            save_env_state(self.save_dir, episode, self.comm.rank, self.envs)
        if self.comm.is_main:
            self.policy.save(self.save_dir, episode)
            if getattr(self.all_args, "save_trainer_state", True):
                from ..utils.checkpoint import save_trainer_state
                save_trainer_state(os.path.join(self.save_dir, f"trainer_state_{episode}.pt"), self.policy,
                                   self.trainer, episode)
        self.comm.barrier()

    def resume(self, models_dir=None):
        """Restore the latest complete checkpoint (weights + Adam + ValueNorm + episode + env counters)."""
        from ..utils.checkpoint import latest_checkpoint, load_env_state, load_trainer_state
        models_dir = models_dir or self.save_dir
        ep = latest_checkpoint(models_dir) if models_dir else None
        if ep is None:
            return None
        self.policy.restore(os.path.join(models_dir, f"transformer_{ep}.pt"))
        load_trainer_state(os.path.join(models_dir, f"trainer_state_{ep}.pt"), self.policy, self.trainer)
        self._resumed = load_env_state(models_dir, ep, self.comm.rank, self.envs)
        self.start_episode = ep + 1
        if self.comm.is_main:
            print(f"[resume] restored episode {ep} from {models_dir}")
        return ep

    # ---------------------------------------------------------------------------------------- eval
    def decide(self, obs, share, ava, stride):
        return self.policy.get_actions(None, obs, ava, deterministic=True, stride=stride)[1]

    @torch.no_grad()
    def eval(self, total_num_steps=0, stride=None, n_steps=None):
        stride = self.eval_stride if stride is None else stride
        env = self.eval_envs
        obs, share, ava = env.reset()
        E = env.E
        n_steps = n_steps or max(1, self.all_args.eval_episodes * 2)
        ep_r = torch.zeros(E, device=self.device)
        ep_d = torch.zeros(E, device=self.device)
        ep_p = torch.zeros(E, device=self.device)
        stats = torch.zeros(4, device=self.device, dtype=torch.float64)
        times = []
        for _ in range(n_steps):
            if self.device.type == "cuda":
                torch.cuda.synchronize()
            t0 = time.time()
            actions = self.decide(obs, share, ava, stride)
            if self.device.type == "cuda":
                torch.cuda.synchronize()
            times.append(time.time() - t0)
            obs, share, reward, done, delay, pay, ava = env.step(actions)
            ep_r += reward
            ep_d += delay
            ep_p += pay
            dd = done.double()
            stats += torch.stack([dd.sum(), (ep_r.double() * dd).sum(), (ep_d.double() * dd).sum(),
                                  (ep_p.double() * dd).sum()])
            keep = (~done).float()
            ep_r *= keep
            ep_d *= keep
            ep_p *= keep
        self.comm.all_reduce_sum_(stats)
        n = max(float(stats[0]), 1.0)
        res = (float(stats[1]) / n, float(stats[2]) / n, float(stats[3]) / n, float(np.mean(times)))
        if self.comm.is_main:
            print(f"eval average episode rewards: {res[0]}, delays: {res[1]}, payments: {res[2]}.")
            print("Inference time: ", res[3])
            self.writter.add_scalars("eval", {"average_episode_rewards": res[0], "average_episode_delays": res[1],
                                              "average_episode_payments": res[2], "inference_time": res[3]},
                                     total_num_steps)
        return res
