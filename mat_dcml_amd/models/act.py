"""MAT action sampling: autoregressive decode (rollout / eval) and teacher-forced evaluation (training).

Behavioural contract — reference ``mat_src/mat/algorithms/utils/transformer_act.py``:

* ``Semi_Discrete`` (DCML): agents ``0..L-2`` are Categorical(act_dim) over availability-masked logits
  (``logit[ava == 0] = -1e10``, ``:8-22``), the last agent is Normal(mean = its 2 logits,
  std = sigmoid(log_std)·0.5) of which column 1 is the ratio action (``:24-28,91-98``).
* Stochastic decode is the exact per-agent loop (``:76-99``) — here with a KV cache, O(L) rows instead of
  O(L) full passes (exact: App. B.2).
* Deterministic decode is "Batch MAT Decision-Making" (``:37-75``): blocks [0,1), [1,1+s), …, capped at the
  discrete-agent count, then one block per continuous agent; agents inside a block see zero rows for their
  in-block predecessors.  Reproduced exactly: each pass recomputes the rows whose inputs changed since the
  previous pass plus the new block.
* Teacher-forced ``parallel_act`` (``:103-129,176-189,219-232,285-322``): one decoder pass over the shifted
  actions; log-probs and entropies per agent.
* ``Discrete`` deterministic: the reference writes the one-hot into row ``i+start`` instead of ``i+start+1``
  and hard-codes stride 4 (``:153,156``); fixed here.

Random numbers come in explicitly (``rand = {"u": (B,L) uniforms, "n": (B,L,act_dim) normals}``) so the torch
path and the HIP decode kernel (``ops/mat_fused.py``) can be compared draw for draw.  Categorical sampling is
inverse-CDF on ``u``; Normal sampling is ``mean + std * n``.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

LOG_SQRT_2PI = 0.5 * math.log(2 * math.pi)
MASK_LOGIT = -1e10


def n_discrete_agents(model, L):
    if model.action_type == "Semi_Discrete":
        return L + model.semi_index if model.semi_index < 0 else model.semi_index
    if model.action_type == "Discrete":
        return L
    return 0


def _masked(logit, ava):
    if ava is None:
        return logit
    return logit.masked_fill(ava == 0, MASK_LOGIT)


def _cat_sample(logit, u, deterministic):
    """Inverse-CDF categorical sample; returns (action long, log_prob)."""
    logp_all = torch.log_softmax(logit.float(), -1)
    if deterministic:
        a = logp_all.argmax(-1)
    else:
        cdf = torch.cumsum(logp_all.exp(), -1)
        a = (cdf < u.unsqueeze(-1)).sum(-1).clamp(max=logit.shape[-1] - 1)
    return a, logp_all.gather(-1, a.unsqueeze(-1)).squeeze(-1)


def normal_logprob(x, mean, std):
    return -((x - mean) ** 2) / (2 * std * std) - torch.log(std) - LOG_SQRT_2PI


def normal_entropy(std):
    return 0.5 + LOG_SQRT_2PI + torch.log(std)


def philox_rand(B, L, act_dim, k0, k1, ctr, env0, device, normal=True):
    """The decode kernel's in-kernel sampling noise on the host (csrc/mat_decode.hip draw_u / draw_n): Philox4x32-10
    of (env0 + b, row, ctr, P_POLICY + k) with key (k0, k1); u = x word, Normals by Box-Muller (dims 0, 1 from the
    y, z words of block 0; dims 2k, 2k + 1 from the x, y words of block k).  Keyed by the global env id, so the eager
    rollout is independent of how envs are split over ranks too.  ``normal=False`` (Discrete action spaces, which
    never read them): only ``u`` — no Box-Muller blocks."""
    from ..utils import philox as px
    env = torch.arange(B, device=device, dtype=torch.int64).view(B, 1) + int(env0)
    row = torch.arange(L, device=device, dtype=torch.int64).view(1, L)
    r0 = px.philox4x32(env, row, int(ctr), px.P_POLICY, k0, k1)
    u = px.u01_open(r0[0]).float()
    if not normal:
        return {"u": u}
    n = torch.empty(B, L, act_dim, device=device)
    for k in range((act_dim + 1) // 2):
        r = r0 if k == 0 else px.philox4x32(env, row, int(ctr), px.P_POLICY + k, k0, k1)
        b0, b1 = (r[1], r[2]) if k == 0 else (r[0], r[1])
        rad = torch.sqrt(-2.0 * torch.log(px.u01_open(b0)))
        th = 6.283185307179586 * px.u01_open(b1)
        n[:, :, 2 * k] = (rad * torch.cos(th)).float()
        if 2 * k + 1 < act_dim:
            n[:, :, 2 * k + 1] = (rad * torch.sin(th)).float()
    return {"u": u, "n": n}


def make_rand(B, L, act_dim, device, generator=None):
    return {"u": torch.rand(B, L, device=device, generator=generator),
            "n": torch.randn(B, L, act_dim, device=device, generator=generator)}


def block_schedule(L, n_disc, stride):
    """Decoder-call blocks of ``transformer_act.py:37-75`` as (start, end) pairs."""
    blocks = []
    s, e = 0, 1
    while True:
        blocks.append((s, e))
        if e >= L:
            break
        if e < n_disc:
            s, e = e, min(e + stride, n_disc)
        else:
            s, e = e, min(e + 1, L)
    return blocks


@torch.no_grad()
def autoregressive_act(model, obs_rep, obs, ava=None, deterministic=False, stride=1, rand=None):
    """Returns actions (B,L,out) float32 and log-probs (B,L,out)."""
    dec = model.decoder
    B, L, D = obs_rep.shape
    A = model.action_dim
    dev = obs_rep.device
    atype = model.action_type
    if rand is None and not deterministic:
        rand = make_rand(B, L, A, dev)
    if rand is None:
        rand = {"u": torch.zeros(B, L, device=dev), "n": torch.zeros(B, L, A, device=dev)}
    n_disc = n_discrete_agents(model, L)
    std = model.action_std() if atype != "Discrete" else None

    if dec.dec_actor:  # MAT-Dec: logits independent of previous actions -> one pass
        logits = dec(None, obs_rep, obs)
        return _heads_from_logits(model, logits, ava, deterministic, rand, n_disc, std)

    if atype == "Available_Continous" or atype == "Available_Continuous":
        return _available_continuous_ar(model, obs_rep, obs, ava, deterministic, rand)

    cont_in = atype in ("Continuous", "Continous")
    in_dim = A if cont_in else A + 1
    shifted = torch.zeros(B, L, in_dim, device=dev, dtype=obs_rep.dtype)
    if not cont_in:
        shifted[:, 0, 0] = 1
    out_dim = A if cont_in else 1
    out_a = torch.zeros(B, L, out_dim, device=dev)
    out_lp = torch.zeros(B, L, out_dim, device=dev)
    cache = dec.new_cache(B, L, dev, obs_rep.dtype)

    def emit(i, logit):
        if i < n_disc:
            a, lp = _cat_sample(_masked(logit, None if ava is None else ava[:, i]), rand["u"][:, i], deterministic)
            out_a[:, i, 0] = a.float()
            out_lp[:, i, 0] = lp
            if i + 1 < L:
                shifted[:, i + 1, 1:] = F.one_hot(a, A).to(shifted.dtype)
        else:
            mean = logit.float()
            x = mean if deterministic else mean + std * rand["n"][:, i]
            lp = normal_logprob(x, mean, std)
            if cont_in:
                out_a[:, i] = x
                out_lp[:, i] = lp
                if i + 1 < L:
                    shifted[:, i + 1] = x.to(shifted.dtype)
            else:
                out_a[:, i, 0] = x[:, -1]          # ratio = column 1 (transformer_act.py:95)
                out_lp[:, i, 0] = lp[:, -1]
                if i + 1 < L:
                    shifted[:, i + 1, 1:] = x.to(shifted.dtype)

    if not deterministic or stride <= 1:
        for i in range(L):
            logit = dec.decode_rows(shifted[:, i:i + 1], obs_rep[:, i:i + 1], cache, i)[:, 0]
            emit(i, logit)
    else:
        prev_s = -1
        for (s, e) in block_schedule(L, n_disc, stride):
            lo = prev_s + 1 if prev_s >= 0 else 0
            lo = min(lo, s)
            logits = dec.decode_rows(shifted[:, lo:e], obs_rep[:, lo:e], cache, lo)
            for i in range(s, e):
                emit(i, logits[:, i - lo])
            prev_s = s
    return out_a, out_lp


def _heads_from_logits(model, logits, ava, deterministic, rand, n_disc, std):
    B, L, A = logits.shape
    out_a = torch.zeros(B, L, 1, device=logits.device)
    out_lp = torch.zeros(B, L, 1, device=logits.device)
    if n_disc > 0:
        lg = _masked(logits[:, :n_disc], None if ava is None else ava[:, :n_disc])
        a, lp = _cat_sample(lg, rand["u"][:, :n_disc], deterministic)
        out_a[:, :n_disc, 0] = a.float()
        out_lp[:, :n_disc, 0] = lp
    if n_disc < L:
        mean = logits[:, n_disc:].float()
        x = mean if deterministic else mean + std * rand["n"][:, n_disc:]
        out_a[:, n_disc:, 0] = x[..., -1]
        out_lp[:, n_disc:, 0] = normal_logprob(x, mean, std)[..., -1]
    return out_a, out_lp


def _available_continuous_ar(model, obs_rep, obs, ava, deterministic, rand, discrete_dim=2):
    """``available_continuous_autoregreesive_act`` (``transformer_act.py:234-283``): per agent a one-hot
    availability choice over the first ``discrete_dim`` logits plus a Normal over the rest."""
    dec = model.decoder
    B, L, _ = obs_rep.shape
    A = model.action_dim
    dev = obs_rep.device
    shifted = torch.zeros(B, L, A + 1, device=dev, dtype=obs_rep.dtype)
    shifted[:, 0, 0] = 1
    out_a = torch.zeros(B, L, A, device=dev)
    out_lp = torch.zeros(B, L, A - discrete_dim + 1, device=dev)
    std = model.action_std()[discrete_dim:]
    cache = dec.new_cache(B, L, dev, obs_rep.dtype)
    for i in range(L):
        logit = dec.decode_rows(shifted[:, i:i + 1], obs_rep[:, i:i + 1], cache, i)[:, 0].float()
        lg = _masked(logit[:, :discrete_dim], None if ava is None else ava[:, i, :discrete_dim])
        a, lp = _cat_sample(lg, rand["u"][:, i], deterministic)
        mean = logit[:, discrete_dim:]
        x = mean if deterministic else mean + std * rand["n"][:, i, discrete_dim:]
        act = torch.cat([F.one_hot(a, discrete_dim).float(), x], -1)
        out_a[:, i] = act
        out_lp[:, i] = torch.cat([lp.unsqueeze(-1), normal_logprob(x, mean, std)], -1)
        if i + 1 < L:
            shifted[:, i + 1, 1:] = act.to(shifted.dtype)
    return out_a, out_lp


def shifted_from_actions(model, action):
    """Teacher-forcing decoder input from stored actions (B,L,out)."""
    B, L, _ = action.shape
    A = model.action_dim
    atype = model.action_type
    dev = action.device
    if atype in ("Continuous", "Continous"):
        sh = torch.zeros(B, L, A, device=dev)
        sh[:, 1:] = action[:, :-1]
        return sh
    sh = torch.zeros(B, L, A + 1, device=dev)
    sh[:, 0, 0] = 1
    if atype in ("Available_Continous", "Available_Continuous"):
        sh[:, 1:, 1:] = action[:, :-1]
        return sh
    n_disc = n_discrete_agents(model, L)
    act_all = torch.cat([F.one_hot(action[:, :n_disc, 0].long(), A).float(),
                         action[:, n_disc:, :1].float().expand(B, L - n_disc, A)], 1)
    sh[:, 1:, 1:] = act_all[:, :-1]
    return sh


def heads_logprob_entropy(model, logits, action, ava):
    """Per-agent log-prob and entropy of stored actions given teacher-forced logits (all fp32)."""
    B, L, A = logits.shape
    atype = model.action_type
    logits = logits.float()
    if atype in ("Continuous", "Continous"):
        std = model.action_std()
        return normal_logprob(action, logits, std), normal_entropy(std).expand_as(logits)
    if atype in ("Available_Continous", "Available_Continuous"):
        dd = 2
        lg = _masked(logits[..., :dd], None if ava is None else ava[..., :dd])
        lsm = torch.log_softmax(lg, -1)
        a = action[..., :dd].argmax(-1)
        lp_d = lsm.gather(-1, a.unsqueeze(-1))
        ent_d = -(lsm.exp() * lsm).sum(-1, keepdim=True)
        std = model.action_std()[dd:]
        lp_c = normal_logprob(action[..., dd:], logits[..., dd:], std)
        return torch.cat([lp_d, lp_c], -1), torch.cat([ent_d, normal_entropy(std).expand_as(lp_c)], -1)
    n_disc = n_discrete_agents(model, L)
    lg = _masked(logits[:, :n_disc], None if ava is None else ava[:, :n_disc])
    lsm = torch.log_softmax(lg, -1)
    a = action[:, :n_disc, 0].long()
    lp = lsm.gather(-1, a.unsqueeze(-1))
    p = lsm.exp()
    ent = -(p * lsm).sum(-1, keepdim=True)
    if n_disc == L:
        return lp, ent
    std = model.action_std()
    mean = logits[:, n_disc:]
    x = action[:, n_disc:, :1].float()
    lp_c = normal_logprob(x, mean, std)[..., -1:]
    ent_c = normal_entropy(std)[-1:].expand(B, L - n_disc, 1)
    return torch.cat([lp, lp_c], 1), torch.cat([ent, ent_c], 1)


def parallel_act(model, obs_rep, obs, action, ava=None):
    """Teacher-forced (log_prob, entropy), each (B, L, out)."""
    dec = model.decoder
    if dec.dec_actor:
        logits = dec(None, obs_rep, obs)
    else:
        logits = dec(shifted_from_actions(model, action).to(obs_rep.dtype), obs_rep, obs)
    return heads_logprob_entropy(model, logits, action, ava)
