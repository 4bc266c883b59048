"""Multi-Agent Transformer (MAT) — encoder/decoder policy with a reference-identical ``state_dict``.

Architecture contract (reference ``mat_src/mat/algorithms/mat/algorithm/ma_transformer.py``):

* ``Encoder`` (``:119-154``): x = GELU(W·LN(obs)+b); rep = blocks(LN(x)); v = head(rep).
  ``EncodeBlock`` (``:72-92``) is post-LN, non-causal MHA + 1x MLP.
* ``Decoder`` (``:157-230``): x = LN(GELU(W_a·shifted_action)); ``DecodeBlock`` (``:95-116``):
  x = LN1(x + causalMHA(x)); x = LN2(rep + causalMHA(q=rep, k=x, v=x)); x = LN3(x + MLP(x)); logits = head(x).
* Parameter names, shapes and construction ORDER match the reference, so ``torch.manual_seed(s)`` gives
  bit-identical orthogonal initialisation and ``transformer_{ep}.pt`` files interoperate both ways
  (the ``attn*.mask`` buffers (1,1,L+1,L+1) and the unused ``state_encoder`` / ``decoder.obs_encoder`` are kept).

Compute paths:
* ``MultiAgentTransformer.forward`` / ``encode`` / ``decode_full`` — plain PyTorch math (fp32 or bf16 autocast);
  this is the CPU path and the numerics oracle for the HIP kernels.
* ``mat_dcml_amd.ops.mat_fused`` — hand-written CDNA4 kernels (fused encoder, teacher-forced decoder,
  persistent KV-cached autoregressive decode) that read the same parameters.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.linear import Linear

NORMAL_STD = 0.5  # transformer_act.py:6


def _init(module: nn.Module, gain: float = 0.01, activate: bool = False):
    if activate:
        gain = nn.init.calculate_gain("relu")
    nn.init.orthogonal_(module.weight.data, gain=gain)
    if module.bias is not None:
        nn.init.constant_(module.bias.data, 0)
    return module


class SelfAttention(nn.Module):
    """Multi-head attention with separate K/Q/V/proj linears (``ma_transformer.py:24-69``)."""

    def __init__(self, n_embd, n_head, n_agent, masked=False):
        super().__init__()
        assert n_embd % n_head == 0
        self.masked = masked
        self.n_head = n_head
        self.key = _init(Linear(n_embd, n_embd))
        self.query = _init(Linear(n_embd, n_embd))
        self.value = _init(Linear(n_embd, n_embd))
        self.proj = _init(Linear(n_embd, n_embd))
        self.register_buffer("mask", torch.tril(torch.ones(n_agent + 1, n_agent + 1)).view(1, 1, n_agent + 1, n_agent + 1))

    def forward(self, key, value, query):
        B, L, D = query.shape
        H = self.n_head
        k = self.key(key).view(B, L, H, D // H).transpose(1, 2)
        q = self.query(query).view(B, L, H, D // H).transpose(1, 2)
        v = self.value(value).view(B, L, H, D // H).transpose(1, 2)
        att = (q @ k.transpose(-2, -1)) * (1.0 / math.sqrt(D // H))
        if self.masked:
            causal = torch.ones(L, L, dtype=torch.bool, device=att.device).tril()
            att = att.masked_fill(~causal, float("-inf"))
        att = torch.softmax(att.float(), dim=-1).to(v.dtype)
        y = (att @ v).transpose(1, 2).reshape(B, L, D)
        return self.proj(y)


class EncodeBlock(nn.Module):
    def __init__(self, n_embd, n_head, n_agent):
        super().__init__()
        self.ln1 = nn.LayerNorm(n_embd)
        self.ln2 = nn.LayerNorm(n_embd)
        self.attn = SelfAttention(n_embd, n_head, n_agent, masked=False)
        self.mlp = nn.Sequential(_init(Linear(n_embd, n_embd), activate=True), nn.GELU(),
                                 _init(Linear(n_embd, n_embd)))

    def forward(self, x):
        x = self.ln1(x + self.attn(x, x, x))
        return self.ln2(x + self.mlp(x))


class DecodeBlock(nn.Module):
    def __init__(self, n_embd, n_head, n_agent):
        super().__init__()
        self.ln1 = nn.LayerNorm(n_embd)
        self.ln2 = nn.LayerNorm(n_embd)
        self.ln3 = nn.LayerNorm(n_embd)
        self.attn1 = SelfAttention(n_embd, n_head, n_agent, masked=True)
        self.attn2 = SelfAttention(n_embd, n_head, n_agent, masked=True)
        self.mlp = nn.Sequential(_init(Linear(n_embd, n_embd), activate=True), nn.GELU(),
                                 _init(Linear(n_embd, n_embd)))

    def forward(self, x, rep_enc):
        x = self.ln1(x + self.attn1(x, x, x))
        x = self.ln2(rep_enc + self.attn2(key=x, value=x, query=rep_enc))
        return self.ln3(x + self.mlp(x))


class Encoder(nn.Module):
    def __init__(self, state_dim, obs_dim, n_block, n_embd, n_head, n_agent, encode_state, n_objective=1):
        super().__init__()
        self.state_dim, self.obs_dim, self.n_embd, self.n_agent = state_dim, obs_dim, n_embd, n_agent
        self.encode_state = encode_state
        self.state_encoder = nn.Sequential(nn.LayerNorm(state_dim), _init(Linear(state_dim, n_embd), activate=True), nn.GELU())
        self.obs_encoder = nn.Sequential(nn.LayerNorm(obs_dim), _init(Linear(obs_dim, n_embd), activate=True), nn.GELU())
        self.ln = nn.LayerNorm(n_embd)
        self.blocks = nn.Sequential(*[EncodeBlock(n_embd, n_head, n_agent) for _ in range(n_block)])
        self.head = nn.Sequential(_init(Linear(n_embd, n_embd), activate=True), nn.GELU(), nn.LayerNorm(n_embd),
                                  _init(Linear(n_embd, n_objective)))

    def forward(self, state, obs):
        x = self.state_encoder(state) if self.encode_state else self.obs_encoder(obs)
        rep = self.blocks(self.ln(x))
        return self.head(rep), rep


class Decoder(nn.Module):
    def __init__(self, obs_dim, action_dim, n_block, n_embd, n_head, n_agent, action_type="Discrete",
                 dec_actor=False, share_actor=False):
        super().__init__()
        self.action_dim, self.n_embd = action_dim, n_embd
        self.dec_actor, self.share_actor, self.action_type = dec_actor, share_actor, action_type
        if action_type != "Discrete":
            self.log_std = nn.Parameter(torch.ones(action_dim))
        if dec_actor:
            def actor():
                return nn.Sequential(nn.LayerNorm(obs_dim), _init(Linear(obs_dim, n_embd), activate=True), nn.GELU(),
                                     nn.LayerNorm(n_embd), _init(Linear(n_embd, n_embd), activate=True), nn.GELU(),
                                     nn.LayerNorm(n_embd), _init(Linear(n_embd, action_dim)))
            self.mlp = actor() if share_actor else nn.ModuleList([actor() for _ in range(n_agent)])
        else:
            # Available_Continuous feeds the same (A+1)-wide shifted input as the discrete types (start flag +
            # action vector, transformer_act.py:235-237, :280-281); the reference builds Linear(A, 64) for it
            # (ma_transformer.py:193-197), which cannot take that input — the first decode step fails there
            if action_type in ("Discrete", "Semi_Discrete", "Available_Continuous", "Available_Continous"):
                self.action_encoder = nn.Sequential(_init(Linear(action_dim + 1, n_embd, bias=False), activate=True), nn.GELU())
            else:
                self.action_encoder = nn.Sequential(_init(Linear(action_dim, n_embd), activate=True), nn.GELU())
            self.obs_encoder = nn.Sequential(nn.LayerNorm(obs_dim), _init(Linear(obs_dim, n_embd), activate=True), nn.GELU())
            self.ln = nn.LayerNorm(n_embd)
            self.blocks = nn.Sequential(*[DecodeBlock(n_embd, n_head, n_agent) for _ in range(n_block)])
            self.head = nn.Sequential(_init(Linear(n_embd, n_embd), activate=True), nn.GELU(), nn.LayerNorm(n_embd),
                                      _init(Linear(n_embd, action_dim)))

    def zero_std(self):
        if self.action_type != "Discrete":
            self.log_std.data.zero_()

    def forward(self, action, obs_rep, obs):
        if self.dec_actor:
            if self.share_actor:
                return self.mlp(obs)
            return torch.stack([m(obs[:, n]) for n, m in enumerate(self.mlp)], 1)
        x = self.ln(self.action_encoder(action))
        for block in self.blocks:
            x = block(x, obs_rep)
        return self.head(x)

    # ------------------------------------------------------------- KV-cached incremental decode (torch path)
    def new_cache(self, B, L, device, dtype):
        nb = len(self.blocks)
        return torch.zeros(nb, 4, B, L, self.n_embd, device=device, dtype=dtype)  # [blk][k1,v1,k2,v2]

    def decode_rows(self, act_rows, rep_rows, cache, lo):
        """Compute decoder rows [lo, lo+R) given their shifted-action inputs and encoder reps.

        ``cache`` holds, per block, the self-attention K/V and cross-attention K/V of rows < lo (exact: row i
        depends only on shifted actions 0..i); rows [lo, lo+R) are (over)written.
        """
        B, R, _ = act_rows.shape
        D = self.n_embd
        hi = lo + R
        x = self.ln(self.action_encoder(act_rows))
        for b, blk in enumerate(self.blocks):
            a1, a2 = blk.attn1, blk.attn2
            cache[b, 0, :, lo:hi] = a1.key(x)
            cache[b, 1, :, lo:hi] = a1.value(x)
            y = _cached_attn(a1.query(x), cache[b, 0, :, :hi], cache[b, 1, :, :hi], a1.n_head, lo)
            x = blk.ln1(x + a1.proj(y))
            cache[b, 2, :, lo:hi] = a2.key(x)
            cache[b, 3, :, lo:hi] = a2.value(x)
            y = _cached_attn(a2.query(rep_rows), cache[b, 2, :, :hi], cache[b, 3, :, :hi], a2.n_head, lo)
            x = blk.ln2(rep_rows + a2.proj(y))
            x = blk.ln3(x + blk.mlp(x))
        return self.head(x)


def _cached_attn(q, k, v, H, lo):
    """Causal attention of query rows [lo, lo+R) over key rows [0, lo+R)."""
    B, R, D = q.shape
    T = k.shape[1]
    hs = D // H
    qh = q.view(B, R, H, hs).transpose(1, 2)
    kh = k.reshape(B, T, H, hs).transpose(1, 2)
    vh = v.reshape(B, T, H, hs).transpose(1, 2)
    att = (qh @ kh.transpose(-2, -1)) * (1.0 / math.sqrt(hs))
    rows = torch.arange(lo, lo + R, device=q.device).view(R, 1)
    cols = torch.arange(T, device=q.device).view(1, T)
    att = att.masked_fill(cols > rows, float("-inf"))
    att = torch.softmax(att.float(), -1).to(vh.dtype)
    return (att @ vh).transpose(1, 2).reshape(B, R, D)


class MultiAgentTransformer(nn.Module):
    """``ma_transformer.py:233-339`` with device-tensor inputs (no numpy round trips)."""

    def __init__(self, state_dim, obs_dim, action_dim, n_agent, n_block=2, n_embd=64, n_head=2, encode_state=False,
                 device=torch.device("cpu"), action_type="Discrete", dec_actor=False, share_actor=False, semi_index=-1,
                 n_objective=1):
        super().__init__()
        self.n_agent, self.action_dim, self.action_type = n_agent, action_dim, action_type
        self.semi_index = semi_index if semi_index is not None else -1
        self.n_embd, self.n_head, self.n_block = n_embd, n_head, n_block
        self.dec_actor = dec_actor
        self.n_objective = n_objective
        self.encoder = Encoder(state_dim, obs_dim, n_block, n_embd, n_head, n_agent, encode_state, n_objective)
        self.decoder = Decoder(obs_dim, action_dim, n_block, n_embd, n_head, n_agent, action_type,
                               dec_actor=dec_actor, share_actor=share_actor)
        self.to(device)

    @property
    def device(self):
        return self.decoder.ln.weight.device if hasattr(self.decoder, "ln") else next(self.parameters()).device

    def zero_std(self):
        self.decoder.zero_std()

    def action_std(self):
        return torch.sigmoid(self.decoder.log_std) * NORMAL_STD

    def forward(self, state, obs, action, available_actions=None):
        """Teacher-forced log-prob / value / entropy (``ma_transformer.py:257-295``)."""
        from . import act
        v_loc, obs_rep = self.encoder(state, obs)
        logp, entropy = act.parallel_act(self, obs_rep, obs, action, available_actions)
        return logp, v_loc, entropy

    def get_actions(self, state, obs, available_actions=None, deterministic=False, stride=1, rand=None):
        from . import act
        v_loc, obs_rep = self.encoder(state, obs)
        a, logp = act.autoregressive_act(self, obs_rep, obs, available_actions, deterministic, stride, rand)
        return a, logp, v_loc

    def get_values(self, state, obs, available_actions=None):
        v_loc, _ = self.encoder(state, obs)
        return v_loc
