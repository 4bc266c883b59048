"""RL math ops with a HIP fast path and a PyTorch reference path.

* ``gae`` — GAE(γ, λ) reverse scan over T on ValueNorm-denormalised values
  (reference ``mat_src/mat/utils/shared_buffer.py:207-238``).  HIP: ``gae_reverse_scan`` in ``csrc/rl_ops.hip``
  (one lane per (env, agent, objective) sequence, the whole T-loop in registers).
* ``masked_mean_std`` — advantage normalisation statistics over active entries, population std
  (``mat_trainer.py:193-197``: inactive → NaN, nanmean / nanstd).  Returns sums so DP ranks can all-reduce.
"""
from __future__ import annotations

import torch

from . import kernels


def gae_torch(rewards, value_preds, masks, gamma, lam, value_normalizer, adv_out, ret_out):
    T = rewards.shape[0]
    v = value_normalizer.denormalize(value_preds) if value_normalizer is not None else value_preds
    g = torch.zeros_like(rewards[0])
    for t in reversed(range(T)):
        delta = rewards[t] + gamma * v[t + 1] * masks[t + 1] - v[t]
        g = delta + gamma * lam * masks[t + 1] * g
        adv_out[t] = g
        ret_out[t] = g + v[t]


GAE_MULTI_OBJECTIVE = True   # the HIP scan takes per-objective ValueNorm statistics (mo/dmo buffers)


def gae(rewards, value_preds, masks, gamma, lam, value_normalizer, adv_out, ret_out):
    n_obj = rewards.shape[-1]
    if kernels.use_hip(rewards) and value_preds.shape[-1] == n_obj and masks.shape[-1] == 1:
        if value_normalizer is not None:
            mean, var = value_normalizer.running_mean_var()
            mean, var = mean.reshape(-1).float(), var.reshape(-1).float()
            if mean.numel() == 1 and n_obj > 1:
                mean, var = mean.expand(n_obj), var.expand(n_obj)
            if mean.numel() != n_obj:
                raise ValueError(f"ValueNorm has {mean.numel()} objectives, rewards {n_obj}")
            mv = torch.cat([mean, var.sqrt()]).contiguous()
        else:
            mv = torch.cat([torch.zeros(n_obj, device=rewards.device), torch.ones(n_obj, device=rewards.device)])
        kernels.gae_reverse_scan(rewards, value_preds, masks, mv, gamma, lam, adv_out, ret_out)
        return
    gae_torch(rewards, value_preds, masks, gamma, lam, value_normalizer, adv_out, ret_out)


def masked_sums(x, mask):
    """(sum, sum_sq, count) over entries with mask != 0, packed in one fp64 tensor (for one all-reduce)."""
    m = (mask != 0).to(torch.float64).expand_as(x)
    xd = x.to(torch.float64) * m
    return torch.stack([xd.sum(), (xd * xd).sum(), m.sum()])


def normalize_from_sums(x, sums, eps=1e-5):
    s, sq, n = sums[0], sums[1], sums[2].clamp(min=1)
    mean = s / n
    var = (sq / n - mean * mean).clamp(min=0)
    return ((x - mean.float()) / (var.sqrt().float() + eps))
