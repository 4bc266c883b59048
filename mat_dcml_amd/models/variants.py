"""MAT ablation variants: encoder-only, decoder-only and GRU (``--algorithm_name mat_encoder|mat_decoder|mat_gru``).

Architectures follow the reference modules (parameter names kept, so their state_dicts line up):

* ``MultiAgentEncoder`` — ``mat_src/mat/algorithms/mat/algorithm/mat_encoder.py:88-240``: the MAT encoder plus an
  ``act_head`` producing every agent's logits in ONE pass (no autoregression); value from ``head``.
* ``MultiAgentDecoder`` — ``mat_decoder.py:143-297``: no encoder; the decoder's own ``obs_encoder(obs)`` is the
  cross-attention query, the value comes from ``val_head`` on the final decoder activations (so it depends on
  the shifted actions, as in the reference's last autoregressive pass).
* ``MultiAgentGRU`` — ``mat_gru.py:20-188``: 2-layer GRUs over the agent axis in place of attention; the decoder
  input is ``LN(action_embedding + obs_rep)``.

All three are broken on DCML in the reference (``get_actions`` rejects the ``stride`` kwarg the policy passes,
SURVEY.md C11-C13).  Here they take the same ``(state, obs, action, ava)`` / ``get_actions(..., stride, rand)``
interface as ``MultiAgentTransformer`` and reuse the shared action machinery in ``models/act.py``: Semi_Discrete
heads (Categorical workers + Normal ratio agent), exact batch decision ``stride`` blocks, teacher-forced
evaluation.  The decoder-only model reuses the KV-cached incremental decode; the GRU decoder decodes
incrementally by carrying per-row hidden states (row i depends only on rows <= i, like the causal decoder), so
both are O(L) per decision.  ``state_dim`` is fixed to 37 as in the reference (the state input is unused).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import act as act_mod
from .mat import NORMAL_STD, Decoder, Encoder, _init
from ..ops.linear import Linear

STATE_DIM_UNUSED = 37   # mat_encoder.py:160, mat_gru.py:121


class _VariantBase(nn.Module):
    semi_index = -1
    dec_actor = False

    def action_std(self):
        return torch.sigmoid(self._log_std()) * NORMAL_STD

    def _log_std(self):
        return self.decoder.log_std

    def zero_std(self):
        with torch.no_grad():
            if self.action_type != "Discrete":
                self._log_std().zero_()

    @property
    def device(self):
        return next(self.parameters()).device


# ---------------------------------------------------------------------------------------------- encoder only
class _EncoderWithActHead(Encoder):
    def __init__(self, obs_dim, action_dim, n_block, n_embd, n_head, n_agent, encode_state, action_type, n_objective):
        super().__init__(STATE_DIM_UNUSED, obs_dim, n_block, n_embd, n_head, n_agent, encode_state, n_objective)
        self.act_head = nn.Sequential(_init(Linear(n_embd, n_embd), activate=True), nn.GELU(), nn.LayerNorm(n_embd),
                                      _init(Linear(n_embd, action_dim)))
        if action_type != "Discrete":
            self.log_std = nn.Parameter(torch.ones(action_dim))


class _HeadOnlyDecoder:
    """Decoder facade for act.py: logits = act_head(rep), independent of previous actions (one pass)."""
    dec_actor = True

    def __init__(self, enc):
        self._enc = enc

    def __call__(self, action, obs_rep, obs):
        return self._enc.act_head(obs_rep)


class MultiAgentEncoder(_VariantBase):
    def __init__(self, state_dim, obs_dim, action_dim, n_agent, n_block=2, n_embd=64, n_head=2, encode_state=False,
                 device=torch.device("cpu"), action_type="Discrete", dec_actor=False, share_actor=False,
                 semi_index=-1, n_objective=1):
        super().__init__()
        self.n_agent, self.action_dim, self.action_type = n_agent, action_dim, action_type
        self.semi_index = semi_index if semi_index is not None else -1
        self.encoder = _EncoderWithActHead(obs_dim, action_dim, n_block, n_embd, n_head, n_agent, False,
                                           action_type, n_objective)
        object.__setattr__(self, "decoder", _HeadOnlyDecoder(self.encoder))   # not a submodule: no duplicate keys
        self.to(device)

    def _log_std(self):
        return self.encoder.log_std

    def _enc(self, obs):
        return self.encoder(None, obs)

    def forward(self, state, obs, action, available_actions=None):
        v, rep = self._enc(obs)
        lp, ent = act_mod.parallel_act(self, rep, obs, action, available_actions)
        return lp, v, ent

    def get_actions(self, state, obs, available_actions=None, deterministic=False, stride=1, rand=None):
        v, rep = self._enc(obs)
        a, lp = act_mod.autoregressive_act(self, rep, obs, available_actions, deterministic, stride, rand)
        return a, lp, v

    def get_values(self, state, obs, available_actions=None):
        return self._enc(obs)[0]


# ---------------------------------------------------------------------------------------------- decoder only
class _ValueDecoder(Decoder):
    def __init__(self, obs_dim, action_dim, n_block, n_embd, n_head, n_agent, action_type, n_objective):
        super().__init__(obs_dim, action_dim, n_block, n_embd, n_head, n_agent, action_type)
        self.val_head = nn.Sequential(_init(Linear(n_embd, n_embd), activate=True), nn.GELU(), nn.LayerNorm(n_embd),
                                      _init(Linear(n_embd, n_objective)))

    def features(self, action, obs_rep):
        x = self.ln(self.action_encoder(action))
        for block in self.blocks:
            x = block(x, obs_rep)
        return x


class MultiAgentDecoder(_VariantBase):
    def __init__(self, state_dim, obs_dim, action_dim, n_agent, n_block=2, n_embd=64, n_head=2, encode_state=False,
                 device=torch.device("cpu"), action_type="Discrete", dec_actor=False, share_actor=False,
                 semi_index=-1, n_objective=1):
        super().__init__()
        self.n_agent, self.action_dim, self.action_type = n_agent, action_dim, action_type
        self.semi_index = semi_index if semi_index is not None else -1
        self.decoder = _ValueDecoder(obs_dim, action_dim, n_block, n_embd, n_head, n_agent, action_type, n_objective)
        self.to(device)

    def _teacher(self, obs, action):
        rep = self.decoder.obs_encoder(obs)
        sh = act_mod.shifted_from_actions(self, action).to(rep.dtype)
        x = self.decoder.features(sh, rep)
        return rep, self.decoder.head(x), self.decoder.val_head(x)

    def forward(self, state, obs, action, available_actions=None):
        _, logits, v = self._teacher(obs, action)
        lp, ent = act_mod.heads_logprob_entropy(self, logits, action, available_actions)
        return lp, v, ent

    def get_actions(self, state, obs, available_actions=None, deterministic=False, stride=1, rand=None):
        rep = self.decoder.obs_encoder(obs)
        a, lp = act_mod.autoregressive_act(self, rep, obs, available_actions, deterministic, stride, rand)
        # value of the final pass, all actions known (mat_decoder.py:24-38 returns the last pass's v_loc)
        x = self.decoder.features(act_mod.shifted_from_actions(self, a).to(rep.dtype), rep)
        return a, lp, self.decoder.val_head(x)

    def get_values(self, state, obs, available_actions=None):
        return self.get_actions(state, obs, available_actions)[2]          # mat_decoder.py:294-297


# ---------------------------------------------------------------------------------------------- GRU
class _GRUEncoder(nn.Module):
    def __init__(self, obs_dim, n_embd, n_objective):
        super().__init__()
        self.state_encoder = nn.Sequential(nn.LayerNorm(STATE_DIM_UNUSED),
                                           _init(Linear(STATE_DIM_UNUSED, n_embd), activate=True), nn.GELU())
        self.obs_encoder = nn.Sequential(nn.LayerNorm(obs_dim), _init(Linear(obs_dim, n_embd), activate=True), nn.GELU())
        self.ln = nn.LayerNorm(n_embd)
        self.gru = nn.GRU(n_embd, n_embd, num_layers=2, batch_first=True)
        self.head = nn.Sequential(_init(Linear(n_embd, n_embd), activate=True), nn.GELU(), nn.LayerNorm(n_embd),
                                  _init(Linear(n_embd, n_objective)))

    def forward(self, state, obs):
        rep, _ = self.gru(self.ln(self.obs_encoder(obs)))
        return self.head(rep), rep


class _GRUDecoder(nn.Module):
    dec_actor = False

    def __init__(self, obs_dim, action_dim, n_embd, action_type):
        super().__init__()
        self.action_dim, self.n_embd, self.action_type = action_dim, n_embd, action_type
        if action_type != "Discrete":
            self.log_std = nn.Parameter(torch.ones(action_dim))
        in_dim = action_dim if action_type in ("Continuous", "Continous") else action_dim + 1
        self.action_encoder = nn.Sequential(_init(Linear(in_dim, n_embd, bias=action_type in ("Continuous", "Continous")),
                                                  activate=True), nn.GELU())
        self.obs_encoder = nn.Sequential(nn.LayerNorm(obs_dim), _init(Linear(obs_dim, n_embd), activate=True), nn.GELU())
        self.ln = nn.LayerNorm(n_embd)
        self.gru = nn.GRU(n_embd, n_embd, num_layers=2, batch_first=True)
        self.head = nn.Sequential(_init(Linear(n_embd, n_embd), activate=True), nn.GELU(), nn.LayerNorm(n_embd),
                                  _init(Linear(n_embd, action_dim)))

    def forward(self, action, obs_rep, obs):
        x, _ = self.gru(self.ln(self.action_encoder(action) + obs_rep))
        return self.head(x)

    # incremental decode: cache[i] = hidden state (layers, B, D) after row i
    def new_cache(self, B, L, device, dtype):
        return torch.zeros(L, 2, B, self.n_embd, device=device, dtype=dtype)

    def decode_rows(self, act_rows, rep_rows, cache, lo):
        h0 = cache[lo - 1] if lo > 0 else torch.zeros_like(cache[0])
        x = self.ln(self.action_encoder(act_rows) + rep_rows)
        out = []
        h = h0.contiguous()
        for r in range(x.shape[1]):
            y, h = self.gru(x[:, r:r + 1], h)
            cache[lo + r] = h
            out.append(y)
        return self.head(torch.cat(out, 1))


class MultiAgentGRU(_VariantBase):
    def __init__(self, state_dim, obs_dim, action_dim, n_agent, n_block=2, n_embd=64, n_head=2, encode_state=False,
                 device=torch.device("cpu"), action_type="Discrete", dec_actor=False, share_actor=False,
                 semi_index=-1, n_objective=1):
        super().__init__()
        self.n_agent, self.action_dim, self.action_type = n_agent, action_dim, action_type
        self.semi_index = semi_index if semi_index is not None else -1
        self.encoder = _GRUEncoder(obs_dim, n_embd, n_objective)
        self.decoder = _GRUDecoder(obs_dim, action_dim, n_embd, action_type)
        self.to(device)

    def forward(self, state, obs, action, available_actions=None):
        v, rep = self.encoder(None, obs)
        lp, ent = act_mod.parallel_act(self, rep, obs, action, available_actions)
        return lp, v, ent

    def get_actions(self, state, obs, available_actions=None, deterministic=False, stride=1, rand=None):
        v, rep = self.encoder(None, obs)
        a, lp = act_mod.autoregressive_act(self, rep, obs, available_actions, deterministic, stride, rand)
        return a, lp, v

    def get_values(self, state, obs, available_actions=None):
        return self.encoder(None, obs)[0]


VARIANTS = {"mat_encoder": MultiAgentEncoder, "mat_decoder": MultiAgentDecoder, "mat_gru": MultiAgentGRU}


def build_variant(name, share_obs_dim, obs_dim, act_dim, num_agents, args, device, action_type, semi_index):
    if name not in VARIANTS:
        raise NotImplementedError(f"unknown MAT variant {name!r}")
    return VARIANTS[name](share_obs_dim, obs_dim, act_dim, num_agents, n_block=args.n_block, n_embd=args.n_embd,
                          n_head=args.n_head, encode_state=args.encode_state, device=device, action_type=action_type,
                          semi_index=semi_index, n_objective=getattr(args, "n_objective", 1))
