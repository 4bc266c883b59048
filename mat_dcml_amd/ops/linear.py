"""Token-major Linear with a split-K weight gradient.

MAT's linears are (N tokens x 64) · (64 x 64) with N ≈ 10^5 per minibatch.  For ``dW = dYᵀ·X`` (a 64x64 output
reduced over N) the library picks a single-tile kernel with no K split (measured 328 µs per call, 38% of the
eager update on MI355X, ``profiles/r1_torch_update_kernel_stats.csv``).  Here dW is computed as a batched GEMM over
``S`` token chunks followed by a chunk sum, which fills the chip.  Used by the PyTorch path; the fused HIP
training kernels (``ops/mat_train.py``) accumulate dW in MFMA registers instead.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _wgrad(dy2, x2, chunks):
    N = x2.shape[0]
    S = max(1, min(chunks, N // 512))
    n = (N // S) * S
    g = torch.bmm(dy2[:n].reshape(S, n // S, -1).transpose(1, 2), x2[:n].reshape(S, n // S, -1)).sum(0)
    if n < N:
        g = g + dy2[n:].t() @ x2[n:]
    return g


class _SplitKLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = dy @ w.to(dy.dtype)
        x2 = x.reshape(-1, x.shape[-1])
        dy2 = dy.reshape(-1, dy.shape[-1])
        dw = _wgrad(dy2, x2.to(dy2.dtype), 256).to(w.dtype)
        db = dy2.float().sum(0).to(w.dtype) if ctx.has_b else None
        return dx, dw, db


def linear(x, weight, bias=None):
    if x.is_cuda and torch.is_grad_enabled() and x.numel() // x.shape[-1] >= 8192:
        if torch.is_autocast_enabled("cuda"):
            dt = torch.get_autocast_dtype("cuda")
            with torch.autocast("cuda", enabled=False):
                return _SplitKLinear.apply(x.to(dt), weight.to(dt), None if bias is None else bias.to(dt))
        return _SplitKLinear.apply(x, weight, bias)
    return F.linear(x, weight, bias)


class Linear(torch.nn.Linear):
    """``nn.Linear`` (same parameters / state_dict keys) routed through the split-K weight gradient."""

    def forward(self, x):
        return linear(x, self.weight, self.bias)
