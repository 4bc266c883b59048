"""Device-resident rollout storage for MAT (+ GAE and the whole-sequence minibatch sampler).

Replaces the numpy ``SharedReplayBuffer`` (reference ``mat_src/mat/utils/shared_buffer.py:22-314``):

* Layout (T+1, E, A, ·) in HBM; ``share_obs`` is stored once per env (E, S) instead of tiled per agent
  (the network ignores it) and the never-read ``rnn_states`` are dropped.
* ``compute_returns`` is GAE on ValueNorm-denormalised values (``shared_buffer.py:207-238``); the reverse
  scan runs as one fused HIP kernel when available (``csrc/rl_ops.hip: gae_reverse_scan``).
* ``minibatches`` = ``feed_forward_generator_transformer`` (``:240-314``): randperm over the T·E sequences,
  split into ``num_mini_batch`` chunks, whole agent sequences kept (the agent shuffle is the identity); on the
  HIP path the permutation is one keyed-Feistel launch (``csrc/rl_ops.hip: randperm_kernel``).
* ``save`` / ``load`` write and read a ``.pt`` of tensors (the reference ``load`` opened its file with
  ``"wb"`` and truncated it, ``shared_buffer.py:106`` — fixed).
"""
from __future__ import annotations

import torch


class RolloutBuffer:
    def __init__(self, T, E, A, obs_dim, share_dim, act_dim, act_out=1, logp_dim=1, gamma=0.99, gae_lambda=0.95,
                 use_valuenorm=True, n_objective=1, device="cpu", store_share=True, use_advantage_norm=False):
        self.T, self.E, self.A = T, E, A
        self.gamma, self.gae_lambda = gamma, gae_lambda
        self.use_valuenorm = use_valuenorm
        self.use_advantage_norm = use_advantage_norm   # DMO buffer: GAE in ValueNorm-normalised space
        self.n_objective = n_objective
        dev = torch.device(device)
        f32 = torch.float32
        self.obs = torch.zeros(T + 1, E, A, obs_dim, dtype=f32, device=dev)
        self.share_obs = torch.zeros(T + 1, E, share_dim, dtype=f32, device=dev) if store_share else None
        self.actions = torch.zeros(T, E, A, act_out, dtype=f32, device=dev)
        self.action_log_probs = torch.zeros(T, E, A, logp_dim, dtype=f32, device=dev)
        self.value_preds = torch.zeros(T + 1, E, A, n_objective, dtype=f32, device=dev)
        self.returns = torch.zeros(T + 1, E, A, n_objective, dtype=f32, device=dev)
        self.advantages = torch.zeros(T, E, A, n_objective, dtype=f32, device=dev)
        self.rewards = torch.zeros(T, E, A, n_objective, dtype=f32, device=dev)
        self.masks = torch.ones(T + 1, E, A, 1, dtype=f32, device=dev)
        self.active_masks = torch.ones(T + 1, E, A, 1, dtype=f32, device=dev)
        self.available_actions = torch.ones(T + 1, E, A, act_dim, dtype=f32, device=dev)
        self.step = 0

    def insert(self, share_obs, obs, actions, action_log_probs, value_preds, rewards, masks, active_masks=None,
               available_actions=None):
        t = self.step
        if self.share_obs is not None and share_obs is not None:
            self.share_obs[t + 1].copy_(share_obs if share_obs.dim() == 2 else share_obs[:, 0])
        self.obs[t + 1].copy_(obs)
        self.actions[t].copy_(actions.view_as(self.actions[t]))
        self.action_log_probs[t].copy_(action_log_probs.view_as(self.action_log_probs[t]))
        self.value_preds[t].copy_(value_preds.view_as(self.value_preds[t]))
        self.rewards[t].copy_(rewards.view_as(self.rewards[t]) if rewards.numel() == self.rewards[t].numel()
                              else rewards.view(self.E, 1, -1).expand_as(self.rewards[t]))
        self.masks[t + 1].copy_(masks.view(self.E, -1, 1).expand_as(self.masks[t + 1]))
        if active_masks is not None:
            self.active_masks[t + 1].copy_(active_masks.view(self.E, -1, 1).expand_as(self.active_masks[t + 1]))
        if available_actions is not None:
            self.available_actions[t + 1].copy_(available_actions)
        self.step = (t + 1) % self.T

    def after_update(self):
        for name in ("obs", "masks", "active_masks", "available_actions"):
            buf = getattr(self, name)
            buf[0].copy_(buf[-1])
        if self.share_obs is not None:
            self.share_obs[0].copy_(self.share_obs[-1])

    @torch.no_grad()
    def compute_returns(self, next_value, value_normalizer=None):
        """GAE per objective column.  ``use_advantage_norm`` = the DMO buffer (``dmo_shared_buffer.py:233-280``):
        delta = normalize(r) + γ·v' − v on normalised predictions, returns = denormalize(gae + v) once the
        normaliser has statistics (the raw objectives before that)."""
        vn = value_normalizer if self.use_valuenorm else None
        if not self.use_advantage_norm:
            from ..ops import kernels
            n_obj = self.rewards.shape[-1]
            nv = next_value.reshape(-1)
            if (kernels.use_hip(self.rewards) and self.value_preds.shape[-1] == n_obj and self.masks.shape[-1] == 1
                    and nv.numel() == self.value_preds[-1].numel() and nv.dtype == torch.float32
                    and (vn is None or vn.running_mean.numel() in (1, n_obj))):
                # one launch: V(T) slot copy + ValueNorm statistics + the reverse scan (ops/kernels.gae_reverse_scan_vn)
                kernels.gae_reverse_scan_vn(self.rewards, self.value_preds, self.masks, nv.contiguous(), vn, self.gamma,
                                            self.gae_lambda, self.advantages, self.returns)
                return
        self.value_preds[-1].copy_(next_value.view_as(self.value_preds[-1]))
        if self.use_advantage_norm and vn is not None:
            updated = bool(vn.debiasing_term.reshape(-1)[0] > 0)
            r = vn.normalize(self.rewards)
            g = torch.zeros_like(self.rewards[0])
            for t in reversed(range(self.T)):
                delta = r[t] + self.gamma * self.value_preds[t + 1] * self.masks[t + 1] - self.value_preds[t]
                g = delta + self.gamma * self.gae_lambda * self.masks[t + 1] * g
                self.advantages[t] = g
                self.returns[t] = vn.denormalize(g + self.value_preds[t]) if updated else self.rewards[t]
            return
        from ..ops import rl_ops
        rl_ops.gae(self.rewards, self.value_preds, self.masks, self.gamma, self.gae_lambda,
                   value_normalizer if self.use_valuenorm else None, self.advantages, self.returns)

    def minibatch_indices(self, num_mini_batch, generator=None):
        n = self.T * self.E
        mb = n // num_mini_batch
        from ..ops import kernels
        if kernels.use_hip(self.obs):   # one keyed-Feistel launch instead of torch's ~10-launch radix sort
            perm = kernels.randperm(n, self.obs.device, generator)
        else:
            perm = torch.randperm(n, device=self.obs.device, generator=generator)
        return [perm[i * mb:(i + 1) * mb] for i in range(num_mini_batch)]

    def flat(self, name):
        x = getattr(self, name)
        if name in ("obs", "masks", "active_masks", "available_actions", "value_preds", "returns"):
            x = x[:-1]
        return x.reshape(self.T * self.E, *x.shape[2:])

    def state_dict(self):
        return {k: v for k, v in self.__dict__.items() if isinstance(v, torch.Tensor)} | {"step": self.step}

    def save(self, path):
        torch.save(self.state_dict(), path)

    def load(self, path):
        sd = torch.load(path, map_location=self.obs.device, weights_only=True)
        for k, v in sd.items():
            if k == "step":
                self.step = int(v)
            else:
                getattr(self, k).copy_(v)
