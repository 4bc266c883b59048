"""Agent-batched actor-critic networks for the baseline algorithms (HAPPO, R-MAPPO, IPPO, HATRPO, PPO).

Capability parity with the reference's generic nets:

* ``MLPBase`` / ``MLPLayer`` (``mat_src/mat/algorithms/utils/mlp.py``): optional input LayerNorm, Linear →
  Tanh|ReLU → LayerNorm blocks, orthogonal|xavier init with the activation gain; an ``output`` MLP on top.
* ``RNNLayer`` (``utils/rnn.py``): multi-layer GRU with hidden state reset by ``masks``, LayerNorm on the output.
* ``CNNBase`` (``utils/cnn.py``): conv → ReLU → flatten → Linear for image observations.
* ``ACTLayer`` + distributions (``utils/act.py``, ``utils/distributions.py``): Discrete (Categorical with
  availability masking), Box (DiagGaussian, std = sigmoid(log_std / x_coef) · y_coef), MultiBinary
  (Bernoulli), MultiDiscrete, and the DCML "mixed" single-agent space (W Categorical(2) + a Normal ratio).
* ``PopArt`` output layer (``utils/popart.py``).
* ``R_Actor`` / ``R_Critic`` (``r_mappo/r_actor_critic.py``, ``algorithms/actor_critic.py``).

MI355X design: the reference instantiates one actor and one critic *per agent* and runs them in Python loops
(101 tiny forward passes per env step on DCML).  Here every parameter carries a leading agent axis M and a
layer runs all M agents as ONE batched GEMM (``einsum('bmi,moi->bmo')`` → rocBLAS strided-batched GEMM).  The
per-agent view (``idx=k``) slices agent k's weights, so sequential-update algorithms (HAPPO / HATRPO) still
update one agent at a time with its own optimizer state (``algos/stacked_adam.py``).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Bernoulli, Categorical, Normal, kl_divergence

MASK_LOGIT = -1e10


def _ortho_(w: torch.Tensor, gain: float, orthogonal: bool = True):
    for m in range(w.shape[0]):
        (nn.init.orthogonal_ if orthogonal else nn.init.xavier_uniform_)(w[m], gain=gain)


class SLinear(nn.Module):
    """M independent Linear layers (one per agent).  x: (..., M, in) → (..., M, out); with idx: (..., in)."""

    def __init__(self, M, i, o, gain=1.0, orthogonal=True, bias=True):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(M, o, i))
        _ortho_(self.weight.data, gain, orthogonal)
        self.bias = nn.Parameter(torch.zeros(M, o)) if bias else None

    def forward(self, x, idx=None):
        if idx is None:
            y = torch.einsum("...mi,moi->...mo", x, self.weight)
            return y + self.bias if self.bias is not None else y
        y = x @ self.weight[idx].t()
        return y + self.bias[idx] if self.bias is not None else y


class SLayerNorm(nn.Module):
    def __init__(self, M, d):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(M, d))
        self.bias = nn.Parameter(torch.zeros(M, d))
        self.d = d

    def forward(self, x, idx=None):
        y = F.layer_norm(x, (self.d,))
        if idx is None:
            return y * self.weight + self.bias
        return y * self.weight[idx] + self.bias[idx]


class MLPLayer(nn.Module):
    def __init__(self, M, in_dim, hidden, layer_N, orthogonal=True, relu=True):
        super().__init__()
        self.act = nn.ReLU() if relu else nn.Tanh()
        gain = nn.init.calculate_gain("relu" if relu else "tanh")
        self.fc = nn.ModuleList([SLinear(M, in_dim if n == 0 else hidden, hidden, gain, orthogonal)
                                 for n in range(layer_N + 1)])
        self.ln = nn.ModuleList([SLayerNorm(M, hidden) for _ in range(layer_N + 1)])

    def forward(self, x, idx=None):
        for fc, ln in zip(self.fc, self.ln):
            x = ln(self.act(fc(x, idx)), idx)
        return x


class MLPBase(nn.Module):
    def __init__(self, M, in_dim, hidden=64, layer_N=1, orthogonal=True, relu=True, feature_norm=True):
        super().__init__()
        self.feature_norm = SLayerNorm(M, in_dim) if feature_norm else None
        self.mlp = MLPLayer(M, in_dim, hidden, layer_N, orthogonal, relu)
        self.output = MLPLayer(M, hidden, hidden, layer_N, orthogonal, relu)
        self.out_dim = hidden

    def forward(self, x, idx=None):
        if self.feature_norm is not None:
            x = self.feature_norm(x, idx)
        return self.output(self.mlp(x, idx), idx)


class CNNBase(nn.Module):
    """Image observations (C, H, W): conv(k=3) → ReLU → flatten → Linear → ReLU, per agent (shared kernel
    applied with the agent axis folded into the batch; the dense part is agent-batched)."""

    def __init__(self, M, obs_shape, hidden=64, orthogonal=True):
        super().__init__()
        C, H, W = obs_shape
        self.obs_shape = obs_shape
        self.conv = nn.Conv2d(C, hidden // 2, 3)
        nn.init.orthogonal_(self.conv.weight, gain=nn.init.calculate_gain("relu"))
        nn.init.zeros_(self.conv.bias)
        self.fc = SLinear(M, hidden // 2 * (H - 2) * (W - 2), hidden, nn.init.calculate_gain("relu"), orthogonal)
        self.out_dim = hidden

    def forward(self, x, idx=None):
        lead = x.shape[:-1]
        img = x.reshape(-1, *self.obs_shape) / 255.0
        y = F.relu(self.conv(img)).flatten(1)
        return F.relu(self.fc(y.reshape(*lead, -1), idx))


class SGRU(nn.Module):
    """``RNNLayer``: ``recurrent_N``-layer GRU over time with mask resets, then LayerNorm.  Agent-batched weights.

    x: (T, ..., M, H) [or (T, ..., H) with idx]; h0: (..., M, N, H) [or (..., N, H)]; masks: (T, ..., M, 1)."""

    def __init__(self, M, in_dim, hidden, recurrent_N=1, orthogonal=True):
        super().__init__()
        self.N, self.H = recurrent_N, hidden
        self.w_ih = nn.ModuleList([SLinear(M, in_dim if n == 0 else hidden, 3 * hidden, 1.0, orthogonal)
                                   for n in range(recurrent_N)])
        self.w_hh = nn.ModuleList([SLinear(M, hidden, 3 * hidden, 1.0, orthogonal) for _ in range(recurrent_N)])
        self.norm = SLayerNorm(M, hidden)

    def _cell(self, n, x, h, idx):
        gi = self.w_ih[n](x, idx)
        gh = self.w_hh[n](h, idx)
        ir, iz, inn = gi.chunk(3, -1)
        hr, hz, hn = gh.chunk(3, -1)
        r = torch.sigmoid(ir + hr)
        z = torch.sigmoid(iz + hz)
        c = torch.tanh(inn + r * hn)
        return (1 - z) * c + z * h

    def forward(self, x, h0, masks, idx=None):
        hs = [h0[..., n, :] for n in range(self.N)]
        outs = []
        for t in range(x.shape[0]):
            m = masks[t]
            hs = [h * m for h in hs]
            y = x[t]
            for n in range(self.N):
                hs[n] = self._cell(n, y, hs[n], idx)
                y = hs[n]
            outs.append(y)
        return self.norm(torch.stack(outs), idx), torch.stack(hs, -2)


# ------------------------------------------------------------------------------------------ distributions
class Dist:
    """Per-sample action distribution with the reference's reductions (``distributions.py``)."""

    def sample(self): ...
    def mode(self): ...
    def log_prob(self, a): ...
    def entropy(self): ...
    def kl(self, old): ...


class CatDist(Dist):
    def __init__(self, logits):
        self.d = Categorical(logits=logits)

    def sample(self):
        return self.d.sample().unsqueeze(-1).float()

    def mode(self):
        return self.d.probs.argmax(-1, keepdim=True).float()

    def log_prob(self, a):
        return self.d.log_prob(a[..., 0].long()).unsqueeze(-1)

    def entropy(self):
        return self.d.entropy().unsqueeze(-1)

    def kl(self, old):
        return kl_divergence(old.d, self.d).unsqueeze(-1)


class NormalDist(Dist):
    def __init__(self, mean, std):
        self.d = Normal(mean, std.expand_as(mean))

    def sample(self):
        return self.d.sample()

    def mode(self):
        return self.d.mean

    def log_prob(self, a):                       # per dimension (FixedNormal.log_probs)
        return self.d.log_prob(a)

    def entropy(self):
        return self.d.entropy().sum(-1, keepdim=True)

    def kl(self, old):
        return kl_divergence(old.d, self.d).sum(-1, keepdim=True)


class BernDist(Dist):
    def __init__(self, logits):
        self.d = Bernoulli(logits=logits)

    def sample(self):
        return self.d.sample()

    def mode(self):
        return (self.d.probs > 0.5).float()

    def log_prob(self, a):
        return self.d.log_prob(a).sum(-1, keepdim=True)

    def entropy(self):
        return self.d.entropy().sum(-1, keepdim=True)

    def kl(self, old):
        return kl_divergence(old.d, self.d).sum(-1, keepdim=True)


class ProductDist(Dist):
    """Independent components over the last axis (MultiDiscrete, DCML mixed); log-probs summed (``act.py``)."""

    def __init__(self, parts, sizes, ent_scale=1.0, ent_mean_cat=False):
        self.parts, self.sizes = parts, sizes
        self.ent_scale, self.ent_mean_cat = ent_scale, ent_mean_cat

    def sample(self):
        return torch.cat([p.sample() for p in self.parts], -1)

    def mode(self):
        return torch.cat([p.mode() for p in self.parts], -1)

    def log_prob(self, a):
        out, o = [], 0
        for p, s in zip(self.parts, self.sizes):
            out.append(p.log_prob(a[..., o:o + s]).sum(-1, keepdim=True))
            o += s
        return torch.stack(out, 0).sum(0)

    def entropy(self):
        ents = [p.entropy() for p in self.parts]
        if self.ent_mean_cat:   # act.py:186-199: mean of the categorical entropies + the Normal's, each / 0.98
            return (torch.stack(ents[:-1], 0).mean(0) + ents[-1]) * self.ent_scale
        return torch.stack(ents, 0).sum(0)

    def kl(self, old):
        return torch.stack([p.kl(q) for p, q in zip(self.parts, old.parts)], 0).sum(0)


class MultiCatDist(Dist):
    """K categoricals of equal size in one tensor: logits (..., K, n) — the batched form of the mixed head."""

    def __init__(self, logits):
        self.d = Categorical(logits=logits)

    def sample(self):
        return self.d.sample().float()

    def mode(self):
        return self.d.probs.argmax(-1).float()

    def log_prob(self, a):
        return self.d.log_prob(a.long()).sum(-1, keepdim=True)

    def entropy(self):
        return self.d.entropy().mean(-1, keepdim=True)

    def kl(self, old):
        return kl_divergence(old.d, self.d).sum(-1, keepdim=True)


class ACTLayer(nn.Module):
    """Action head for one agent group.  ``space`` = (kind, dims):
    ("discrete", n) | ("box", d) | ("multibinary", d) | ("multidiscrete", [n1, n2, …]) | ("mixed", (K, n, c))."""

    def __init__(self, M, space, hidden, orthogonal=True, gain=0.01, std_x_coef=1.0, std_y_coef=0.5):
        super().__init__()
        self.kind, self.dims = space
        self.std_x, self.std_y = std_x_coef, std_y_coef
        k = self.kind
        if k == "discrete":
            self.out = SLinear(M, hidden, self.dims, gain, orthogonal)
            self.act_dim = 1
        elif k == "box":
            self.out = SLinear(M, hidden, self.dims, gain, orthogonal)
            self.log_std = nn.Parameter(torch.ones(M, self.dims) * std_x_coef)
            self.act_dim = self.dims
        elif k == "multibinary":
            self.out = SLinear(M, hidden, self.dims, gain, orthogonal)
            self.act_dim = self.dims
        elif k == "multidiscrete":
            self.outs = nn.ModuleList([SLinear(M, hidden, n, gain, orthogonal) for n in self.dims])
            self.act_dim = len(self.dims)
        elif k == "mixed":
            K, n, c = self.dims
            self.out = SLinear(M, hidden, K * n + c, gain, orthogonal)
            self.log_std = nn.Parameter(torch.ones(M, c))
            self.act_dim = K + c
        else:
            raise ValueError(k)

    def _std(self, idx):
        ls = self.log_std if idx is None else self.log_std[idx]
        if self.kind == "mixed":
            return torch.sigmoid(ls) * 0.5                      # act.py:115-116
        return torch.sigmoid(ls / self.std_x) * self.std_y     # DiagGaussian

    def dist(self, x, ava=None, idx=None) -> Dist:
        k = self.kind
        if k == "discrete":
            logits = self.out(x, idx)
            if ava is not None:
                logits = logits.masked_fill(ava == 0, MASK_LOGIT)
            return CatDist(logits)
        if k == "box":
            return NormalDist(self.out(x, idx), self._std(idx))
        if k == "multibinary":
            return BernDist(self.out(x, idx))
        if k == "multidiscrete":
            ps = [CatDist(o(x, idx)) for o in self.outs]
            return ProductDist(ps, [1] * len(ps))
        K, n, c = self.dims
        y = self.out(x, idx)
        logits = y[..., :K * n].reshape(*y.shape[:-1], K, n)
        if ava is not None:
            logits = logits.masked_fill(ava[..., :K * n].reshape(logits.shape) == 0, MASK_LOGIT)
        return ProductDist([MultiCatDist(logits), NormalDist(y[..., K * n:], self._std(idx))], [K, c],
                           ent_scale=1 / 0.98, ent_mean_cat=True)


# ------------------------------------------------------------------------------------------ PopArt
class PopArt(nn.Module):
    """Agent-batched PopArt value head (``algorithms/utils/popart.py``): running mean/std of the targets; an
    update rescales the output layer so un-normalised predictions are preserved."""

    def __init__(self, M, hidden, out=1, beta=0.99999, epsilon=1e-5):
        super().__init__()
        self.beta, self.eps = beta, epsilon
        self.lin = SLinear(M, hidden, out, 1.0)
        self.register_buffer("mean", torch.zeros(M, out))
        self.register_buffer("mean_sq", torch.zeros(M, out))
        self.register_buffer("debias", torch.zeros(M, 1))
        self.register_buffer("stddev", torch.ones(M, out))

    def forward(self, x, idx=None):
        return self.lin(x, idx)

    def _mv(self):
        d = self.debias.clamp(min=self.eps)
        mean = self.mean / d
        var = (self.mean_sq / d - mean ** 2).clamp(min=1e-4)
        return mean, var

    @torch.no_grad()
    def update(self, x, idx=None):
        """x: (N, M, out) [or (N, out) for agent idx]."""
        old_mean, old_var = self._mv()
        old_std = old_var.sqrt()
        sl = slice(None) if idx is None else slice(idx, idx + 1)
        xb = x.float().reshape(-1, *(self.mean[sl].shape))
        bm, bsq = xb.mean(0), (xb * xb).mean(0)
        self.mean[sl] = self.mean[sl] * self.beta + bm * (1 - self.beta)
        self.mean_sq[sl] = self.mean_sq[sl] * self.beta + bsq * (1 - self.beta)
        self.debias[sl] = self.debias[sl] * self.beta + (1 - self.beta)
        new_mean, new_var = self._mv()
        new_std = new_var.sqrt()
        self.stddev.copy_(new_std)
        w, b = self.lin.weight.data, self.lin.bias.data
        w[sl] = w[sl] * (old_std[sl] / new_std[sl]).unsqueeze(-1)
        b[sl] = (old_std[sl] * b[sl] + old_mean[sl] - new_mean[sl]) / new_std[sl]

    def normalize(self, x, idx=None):
        mean, var = self._mv()
        if idx is not None:
            mean, var = mean[idx], var[idx]
        return (x - mean) / var.sqrt()

    def denormalize(self, x, idx=None):
        mean, var = self._mv()
        if idx is not None:
            mean, var = mean[idx], var[idx]
        return x * var.sqrt() + mean


# ------------------------------------------------------------------------------------------ actor / critic
class Actor(nn.Module):
    """``R_Actor`` for a group of M agents sharing one observation size and action space."""

    def __init__(self, M, obs_dim, space, args, obs_shape=None):
        super().__init__()
        h = args.hidden_size
        if obs_shape is not None and len(obs_shape) == 3:
            self.base = CNNBase(M, obs_shape, h, args.use_orthogonal)
        else:
            self.base = MLPBase(M, obs_dim, h, args.layer_N, args.use_orthogonal, args.use_ReLU,
                                args.use_feature_normalization)
        self.recurrent = args.use_recurrent_policy or args.use_naive_recurrent_policy
        if self.recurrent:
            self.rnn = SGRU(M, h, h, args.recurrent_N, args.use_orthogonal)
        self.act = ACTLayer(M, space, h, args.use_orthogonal, args.gain, args.std_x_coef, args.std_y_coef)

    def features(self, obs, h0, masks, idx=None):
        """obs (T, ..., in) → features (T, ..., H), h (..., N, H)."""
        x = self.base(obs, idx)
        if self.recurrent:
            return self.rnn(x, h0, masks, idx)
        return x, h0

    def forward(self, obs, h0, masks, ava=None, deterministic=False, idx=None):
        x, h = self.features(obs, h0, masks, idx)
        d = self.act.dist(x, ava, idx)
        a = d.mode() if deterministic else d.sample()
        return a, d.log_prob(a), h

    def evaluate_actions(self, obs, h0, actions, masks, ava=None, idx=None):
        x, _ = self.features(obs, h0, masks, idx)
        d = self.act.dist(x, ava, idx)
        return d.log_prob(actions), d.entropy(), d


class Critic(nn.Module):
    """``R_Critic``: value V(share_obs) per agent, optional GRU, Linear or PopArt output."""

    def __init__(self, M, share_dim, args, popart=False, n_out=1):
        super().__init__()
        h = args.hidden_size
        self.base = MLPBase(M, share_dim, h, args.layer_N, args.use_orthogonal, args.use_ReLU,
                            args.use_feature_normalization)
        self.recurrent = args.use_recurrent_policy or args.use_naive_recurrent_policy
        if self.recurrent:
            self.rnn = SGRU(M, h, h, args.recurrent_N, args.use_orthogonal)
        self.popart = popart
        self.v_out = PopArt(M, h, n_out) if popart else SLinear(M, h, n_out, 1.0, args.use_orthogonal)

    def forward(self, share, h0, masks, idx=None):
        x = self.base(share, idx)
        h = h0
        if self.recurrent:
            x, h = self.rnn(x, h0, masks, idx)
        return self.v_out(x, idx), h


def space_of(act_space):
    """Reference action-space object → (kind, dims) for ``ACTLayer``."""
    cls = act_space.__class__.__name__
    if cls == "Discrete":
        return ("discrete", int(act_space.n))
    if cls == "Box":
        return ("box", int(act_space.shape[0]))
    if cls == "MultiBinary":
        return ("multibinary", int(act_space.shape[0]))
    if cls == "MultiDiscrete":
        return ("multidiscrete", [int(h - l + 1) for l, h in zip(act_space.low, act_space.high)])
    if cls in ("Action_Space", "ActionSpec"):
        if getattr(act_space, "mixed", False) and getattr(act_space, "semi_index", 0) != 0:
            K = int(act_space.high - act_space.low)
            return ("mixed", (K, int(act_space.n), -int(act_space.semi_index)))
        if getattr(act_space, "extra", False) or getattr(act_space, "continuous", False) and not act_space.mixed:
            return ("box", int(act_space.n))
        return ("discrete", int(act_space.n))
    raise ValueError(f"unsupported action space {cls}")


def flat_params(module_params):
    return torch.cat([p.reshape(-1) for p in module_params])


def n_params(m):
    return sum(p.numel() for p in m.parameters())


__all__ = ["SLinear", "SLayerNorm", "MLPLayer", "MLPBase", "CNNBase", "SGRU", "ACTLayer", "PopArt", "Actor",
           "Critic", "space_of", "CatDist", "NormalDist", "BernDist", "ProductDist", "MultiCatDist", "math"]
