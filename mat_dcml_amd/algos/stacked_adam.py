"""Adam over agent-stacked parameters with per-agent state.

The reference gives every agent its own ``torch.optim.Adam`` (``rMAPPOPolicy.py``, ``happo_policy.py``).  With
agent-batched weights (``models/ac.py``) each parameter is (M, ...); this optimizer keeps one step counter per
agent and can update either every agent at once (independent learners: IPPO, R-MAPPO) or a single agent's slice
(sequential learners: HAPPO, HATRPO) — the other agents' weights and moments are untouched, exactly as if they
had separate optimizers.  Per-agent gradient-norm clipping matches ``clip_grad_norm_`` on each agent's own net.
"""
from __future__ import annotations

import torch


class StackedAdam:
    def __init__(self, params, M, lr=1e-3, eps=1e-5, betas=(0.9, 0.999), weight_decay=0.0):
        self.params = [p for p in params if p.requires_grad]
        self.M = M
        self.lr, self.eps, self.betas, self.wd = lr, eps, betas, weight_decay
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        dev = self.params[0].device
        self.t = torch.zeros(M, device=dev)

    def zero_grad(self):
        for p in self.params:
            p.grad = None

    def _view(self, x):
        return x.reshape(self.M, -1)

    def grad_norms(self, idx=None):
        """Per-agent L2 norms of the current gradients: (M,) or scalar for idx."""
        sq = None
        for p in self.params:
            if p.grad is None:
                continue
            g = self._view(p.grad)
            s = (g.float() ** 2).sum(1) if idx is None else (g[idx].float() ** 2).sum()
            sq = s if sq is None else sq + s
        if sq is None:
            return torch.zeros(self.M if idx is None else (), device=self.t.device)
        return sq.sqrt()

    def clip_(self, max_norm, idx=None):
        norms = self.grad_norms(idx)
        scale = (max_norm / (norms + 1e-6)).clamp(max=1.0)
        for p in self.params:
            if p.grad is None:
                continue
            g = self._view(p.grad)
            if idx is None:
                g.mul_(scale.view(self.M, 1))
            else:
                g[idx].mul_(scale)
        return norms

    @torch.no_grad()
    def step(self, idx=None):
        b1, b2 = self.betas
        if idx is None:
            self.t += 1
            bc1 = (1 - b1 ** self.t).view(self.M, 1)
            bc2 = (1 - b2 ** self.t).view(self.M, 1)
        else:
            self.t[idx] += 1
            bc1 = 1 - b1 ** self.t[idx]
            bc2 = 1 - b2 ** self.t[idx]
        for p, m, v in zip(self.params, self.m, self.v):
            if p.grad is None:
                continue
            P, G, Mm, V = self._view(p.data), self._view(p.grad), self._view(m), self._view(v)
            if idx is not None:
                P, G, Mm, V = P[idx], G[idx], Mm[idx], V[idx]
            g = G + self.wd * P if self.wd else G
            Mm.mul_(b1).add_(g, alpha=1 - b1)
            V.mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = (V / bc2).sqrt().add_(self.eps)
            P.sub_(self.lr * (Mm / bc1) / denom)

    def set_lr(self, lr):
        self.lr = lr

    def state_dict(self):
        return {"m": self.m, "v": self.v, "t": self.t, "lr": self.lr}

    def load_state_dict(self, sd):
        for a, b in zip(self.m, sd["m"]):
            a.copy_(b)
        for a, b in zip(self.v, sd["v"]):
            a.copy_(b)
        self.t.copy_(sd["t"])
        self.lr = sd["lr"]
