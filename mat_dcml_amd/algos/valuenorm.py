"""Running mean/variance value normaliser, device resident and data-parallel aware.

Same statistics as the reference ``mat_src/mat/utils/valuenorm.py:8-80`` (β = 0.99999, ε = 1e-5,
debiased, variance clamped at 1e-2) and ``mat_src/mat/utils/popart.py`` (``forward`` = update + normalise),
but ``denormalize`` stays on device (the reference returns numpy and forces ≈1,600 device→host syncs per PPO
iteration) and ``update`` can all-reduce its batch moments so every rank keeps identical
statistics (global-batch semantics under DP).
"""
from __future__ import annotations

import torch
import torch.nn as nn


class ValueNorm(nn.Module):
    def __init__(self, input_shape=1, norm_axes=1, beta=0.99999, per_element_update=False, epsilon=1e-5,
                 device=torch.device("cpu"), comm=None):
        super().__init__()
        self.norm_axes, self.epsilon, self.beta = norm_axes, epsilon, beta
        self.per_element_update = per_element_update
        self.comm = comm
        shape = (input_shape,) if isinstance(input_shape, int) else tuple(input_shape)
        self.register_buffer("running_mean", torch.zeros(shape, device=device))
        self.register_buffer("running_mean_sq", torch.zeros(shape, device=device))
        self.register_buffer("debiasing_term", torch.zeros((), device=device))

    def reset_parameters(self):
        self.running_mean.zero_()
        self.running_mean_sq.zero_()
        self.debiasing_term.zero_()

    def running_mean_var(self):
        d = self.debiasing_term.clamp(min=self.epsilon)
        mean = self.running_mean / d
        var = (self.running_mean_sq / d - mean ** 2).clamp(min=1e-2)
        return mean, var

    @torch.no_grad()
    def update(self, x: torch.Tensor, presummed=None):
        """``presummed`` = (Σx, Σx², n) already reduced over the (global) batch — the data-parallel trainer computes
        every minibatch's moments of an epoch up front and all-reduces them in one message (MATTrainer.train)."""
        if presummed is not None:
            s, sq, n = presummed
            s, sq = s.float().view_as(self.running_mean), sq.float().view_as(self.running_mean)
            n = n.float() if torch.is_tensor(n) else float(n)
            mean, sq_mean = s / n, sq / n
            w = self.beta ** n if self.per_element_update else self.beta
            self.running_mean.mul_(w).add_(mean * (1.0 - w))
            self.running_mean_sq.mul_(w).add_(sq_mean * (1.0 - w))
            self.debiasing_term.mul_(w).add_(1.0 * (1.0 - w))
            return
        # the reference flattens (batch, agents, 1) minibatches to (batch*agents, 1) before updating
        x = x.float().reshape(-1, self.running_mean.numel())
        n = x.shape[0]
        s = x.sum(0).view_as(self.running_mean)
        sq = (x * x).sum(0).view_as(self.running_mean)
        if self.comm is not None and self.comm.world_size > 1:
            packed = torch.cat([s.reshape(-1), sq.reshape(-1),
                                torch.tensor([float(n)], device=x.device)])
            self.comm.all_reduce_sum_(packed)
            k = s.numel()
            s, sq, n = packed[:k].view_as(s), packed[k:2 * k].view_as(sq), packed[2 * k]
        mean, sq_mean = s / n, sq / n
        w = self.beta ** n if self.per_element_update else self.beta
        self.running_mean.mul_(w).add_(mean * (1.0 - w))
        self.running_mean_sq.mul_(w).add_(sq_mean * (1.0 - w))
        self.debiasing_term.mul_(w).add_(1.0 * (1.0 - w))

    def normalize(self, x):
        mean, var = self.running_mean_var()
        return (x - mean) / torch.sqrt(var)

    def denormalize(self, x):
        mean, var = self.running_mean_var()
        return x * torch.sqrt(var) + mean

    def forward(self, x, train=True):
        """PopArt-style call (``mat_src/mat/utils/popart.py:39-64``): update then normalise."""
        if train:
            self.update(x)
        return self.normalize(x)
