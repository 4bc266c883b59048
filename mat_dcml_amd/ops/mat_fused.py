"""Fused HIP MAT paths (gfx950): persistent autoregressive decode (+ fused encoder later in this module).

``get_actions`` runs the MAT rollout policy step as:
  1. the encoder (values + obs representations),
  2. ONE ``mat_decode_persistent`` launch (``csrc/mat_decode.hip``) that decodes all L agents of all envs:
     register-resident decoder weights, LDS KV caches, fused head + masking + sampling + log-probs.
Weights are repacked into the kernel's MFMA B-fragment order once per optimizer step (cached on the model
and keyed by ``model._mdl_version``, bumped by the trainer after every update).
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn.functional as F

from . import kernels
from .kernels import P, check, lib, sig

vp, i32 = ctypes.c_void_p, ctypes.c_int


class DecParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("wpack", "bias", "lnp", "emb", "wh2", "bh2", "stdv", "rep", "ava",
                                               "rnd_u", "rnd_n", "out_a", "out_lp")] + \
               [(n, ctypes.c_int) for n in ("B", "L", "act_dim", "n_disc", "stride", "deterministic", "epw", "rmax", "n_tok",
                                            "tok_start", "tok_zero", "stage", "cont")] + \
               [(n, ctypes.c_void_p) for n in ("wa", "ba", "lnd")] + \
               [("gen", ctypes.c_int)] + [(n, ctypes.c_uint32) for n in ("rk0", "rk1", "rctr")] + \
               [("avail_cont", ctypes.c_int), ("qkv0", ctypes.c_void_p), ("q2pre", ctypes.c_int),
                ("genv0", ctypes.c_uint32), ("hfold", ctypes.c_void_p), ("wfa", ctypes.c_void_p)]


sig("mdl_mat_decode", ctypes.POINTER(DecParams), i32, vp)
sig("mdl_mat_decode_geometry", i32, i32, i32)
sig("mdl_decode_wave_plan", ctypes.POINTER(DecParams), i32)
sig("mdl_decode_spec_plan", ctypes.POINTER(DecParams), i32)
sig("mdl_decode_spec_enable", i32)
sig("mdl_decode_spec_layout", i32)


def _is_cont(model):
    return model.action_type in ("Continuous", "Continous")


def _is_avail_cont(model):
    return model.action_type in ("Available_Continuous", "Available_Continous")


def _n_disc(model, L):
    if model.action_type == "Discrete":
        return L
    if _is_cont(model) or _is_avail_cont(model):
        return 0
    return L + model.semi_index if model.semi_index < 0 else model.semi_index


def unsupported_reasons(model, L=None) -> list:
    """Why the fused decode cannot run this model (empty list = supported)."""
    if not kernels.available():
        return ["HIP library not loaded (kernels=torch or not built)"]
    r = []
    if model.action_type not in ("Semi_Discrete", "Discrete", "Continuous", "Continous", "Available_Continuous",
                                 "Available_Continous"):
        r.append(f"action_type {model.action_type}")
    if _is_avail_cont(model) and model.action_dim < 3:
        r.append(f"Available_Continuous with action_dim {model.action_dim} < 3")
    if model.decoder.dec_actor:
        r.append("dec_actor (mat_dec) has no autoregressive decode")
    if model.n_embd != 64 or model.n_head != 2 or model.n_block not in (1, 2, 3):
        r.append(f"n_embd {model.n_embd} / n_head {model.n_head} / n_block {model.n_block} (kernel: 64 / 2 / 1-3)")
    if model.action_dim > 64:
        r.append(f"action_dim {model.action_dim} > 64")
    if model.action_type == "Semi_Discrete" and model.semi_index != -1:
        r.append(f"semi_index {model.semi_index} != -1")
    if not r and lib().mdl_mat_decode_geometry(model.n_block, L or model.n_agent, 1) <= 0:
        r.append(f"L={L or model.n_agent} does not fit the decode kernel's LDS")
    return r


def supports(model, L=None) -> bool:
    return not unsupported_reasons(model, L)


# One-wave decode (csrc/mat_decode_wave.hip) for one-row token passes; False (or MAT_DCML_DECODE_WAVE=0) keeps every
# decode on the 4-wave kernel (csrc/mat_decode.hip) — the A/B switch and the parity tests' reference.
WAVE_DECODE = os.environ.get("MAT_DCML_DECODE_WAVE", "1") != "0"
# Speculative block 0 on that path (csrc/mat_decode_wave.hip:mat_decode_spec_kernel, n_block 2, act_dim <= 48): block 0
# of the next agent runs for every candidate token on extra waves while the main wave finishes the current agent.
# False (or MAT_DCML_DECODE_SPEC=0) keeps the one-wave kernel — the A/B switch and the parity tests' reference.
SPEC_DECODE = os.environ.get("MAT_DCML_DECODE_SPEC", "1") != "0"
_spec_set = [None]

# envs per decode workgroup: the kernel runs one env per workgroup (its MFMA attention shares the K / V operand
# over the tile's query rows); the geometry query still takes the cap for its signature.
_EPW_CAP = 1


def bump_version(model):
    model._mdl_version = getattr(model, "_mdl_version", 0) + 1


def _bfrag(W):  # (reference packing in torch; the kernels use csrc/rl_ops.hip:pack_weights)
    """torch Linear weight (64 out, 64 in) -> [4 waves][2 ksteps][64 lanes][8] bf16 (lane = 16*(k//8 % 4) + n%16)."""
    return W.detach().reshape(4, 16, 2, 4, 8).permute(0, 2, 3, 1, 4).contiguous().to(torch.bfloat16)


@torch.no_grad()
def decoder_pack(model):
    """Decode-kernel operands: the decoder's B fragments (shared ModelPack), stacked biases / LN params and the
    action-embedding token table, rebuilt once per optimizer step."""
    from . import mat_train
    ver = getattr(model, "_mdl_version", 0)
    cache = getattr(model, "_mdl_dec_pack", None)
    if cache is not None and cache[0] == ver:
        return cache[1]
    mp = mat_train.model_pack(model)
    dec = model.decoder
    lins = mat_train.decoder_linears(model)
    lns = []
    for blk in dec.blocks:
        for ln in (blk.ln1, blk.ln2, blk.ln3):
            lns.append(torch.stack([ln.weight.detach(), ln.bias.detach()]))
    lns.append(torch.stack([dec.head[2].weight.detach(), dec.head[2].bias.detach()]))
    A = model.action_dim
    dev = dec.ln.weight.device
    cont = _is_cont(model)
    avail = _is_avail_cont(model)
    if avail:
        # start row = the [1, 0, ..] token; later rows: W_a[:, 1:] · [onehot(a), x] (no bias), built in-kernel
        toks = torch.zeros(2, A + 1, device=dev)
        toks[0, 0] = 1
        tok_start, tok_zero = 0, 1
    elif cont:
        # continuous inputs: row 0 = the zero start action; later rows are built in-kernel from the sampled vector
        toks = torch.zeros(2, A, device=dev)
        tok_start, tok_zero = 0, 1
    else:
        # token table: 0 = start [1,0..], 1+a = one-hot action a, A+1 = zero row (in-block rows of the stride mode)
        toks = torch.zeros(A + 2, A + 1, device=dev)
        toks[0, 0] = 1
        toks[torch.arange(1, A + 1), torch.arange(1, A + 1)] = 1
        tok_start, tok_zero = 0, A + 1
    emb = dec.ln(dec.action_encoder(toks)).float()
    std = model.action_std().float() if model.action_type != "Discrete" else torch.ones(A, device=dev)
    pack = dict(wpack=mp.decoder_fw, wfa=mp.fa, bias=torch.stack([l.bias.detach() for l in lins]).float().contiguous(),
                lnp=torch.stack(lns).float().contiguous(), emb=emb.contiguous(),
                wh2=dec.head[3].weight.detach().float().contiguous(), bh2=dec.head[3].bias.detach().float().contiguous(),
                stdv=std.contiguous(), n_tok=toks.shape[0], tok_start=tok_start, tok_zero=tok_zero,
                cont=int(cont or avail), avail=int(avail))
    if not (cont or avail) and A <= 64:
        # head LayerNorm folded into the logit GEMV of the fused one-row heads (<= 4 actions: register logits;
        # <= 64: one action per lane): W_h2 diag(gamma), Σ_c W_h2 gamma, W_h2 beta + b_h2 (DecParams.hfold)
        w2, b2 = dec.head[3].weight.detach().float(), dec.head[3].bias.detach().float()
        gam, bet = dec.head[2].weight.detach().float(), dec.head[2].bias.detach().float()
        w2g = w2 * gam.view(1, -1)
        pack["hfold"] = torch.cat([w2g.reshape(-1), w2g.sum(1), w2 @ bet + b2]).contiguous()
    if not (cont or avail):
        # block-0 q / k / v of every token row (the decode's first projection depends only on the previous action)
        a1 = dec.blocks[0].attn1
        pack["qkv0"] = torch.stack([F.linear(emb, lin.weight.float(), lin.bias.float())
                                    for lin in (a1.query, a1.key, a1.value)], 1).contiguous()
    if avail:
        lin = dec.action_encoder[0]
        pack.update(wa=lin.weight.detach()[:, 1:].float().contiguous(), ba=torch.zeros(64, device=dev),
                    lnd=torch.stack([dec.ln.weight.detach(), dec.ln.bias.detach()]).float().contiguous())
    elif cont:
        lin = dec.action_encoder[0]
        pack.update(wa=lin.weight.detach().float().contiguous(), ba=lin.bias.detach().float().contiguous(),
                    lnd=torch.stack([dec.ln.weight.detach(), dec.ln.bias.detach()]).float().contiguous())
    model._mdl_dec_pack = (ver, pack)
    return pack


def refresh_packs(model):
    """Rebuild every weight pack that is keyed by ``model._mdl_version`` (encoder / decoder fragment packs, the decode
    operands, the wide-observation embedding pack) on the CURRENT stream.  A caller that then forks work onto other
    streams (the runner's pipelined rollout) makes them wait on this stream: otherwise the first group would rebuild
    the packs lazily on its own stream after an optimizer step and the other groups, seeing the version already
    current, would read half-written packs."""
    from . import mat_train
    if not next(model.parameters()).is_cuda or kernels.mode() == "torch":
        return
    if supports(model):
        decoder_pack(model)
    if mat_train.encoder_supported(model):
        enc, _, _ = mat_train._state(model, next(model.parameters()).device)
        enc.refresh_packs()


def set_sampling_key(model, seed: int, env0: int = 0):
    """Key the rollout's exploration noise by (seed, GLOBAL env id, decode-call counter): row b of a decode batch draws
    from env ``env0 + b``.  Every rank uses the same key and counter, and the runner passes its env-id offset, so a
    1-GPU run over 2E envs and a 2-GPU run over E envs each produce identical rollouts (the reference
    is irreproducible, DCML_MAT_Train.py:35).  The same draws feed the eager decode (``models/act.philox_rand``)."""
    from ..utils import philox as px
    k0, k1 = px.seed_key((int(seed) * 0x9E3779B1 + 0x51A3) & 0xFFFFFFFFFFFF)
    model._mdl_draw_key = [k0, k1 & 0xFFFFFFFF, 0]
    model._mdl_env0 = int(env0)


def next_draw_key(model):
    """(k0, k1, counter) for the next stochastic decode call; advances the counter.  Without ``set_sampling_key``
    the key comes from torch's CPU generator on first use (torch.manual_seed reproducible)."""
    held = getattr(model, "_mdl_draw_held", None)
    if held is not None:   # inside sampling_group(): every env group of one rollout step shares the step's counter
        return held
    key = getattr(model, "_mdl_draw_key", None)
    if key is None:
        key = [int(x) for x in torch.randint(0, 2 ** 31 - 1, (2,))] + [0]
        model._mdl_draw_key = key
    k0, k1, c = key
    key[2] = (c + 1) & 0xFFFFFFFF
    return k0, k1, c


class sampling_group:
    """Decode calls of ONE rollout step made per env group (runner ``rollout_groups``): the groups share the
    step's draw counter (taken once, ``hold``) and each names its first global env id, so the groups' draws are
    the ones a single call over all envs makes."""

    def __init__(self, model):
        self.model = model
        self.env0 = int(getattr(model, "_mdl_env0", 0))
        self.has_env0 = hasattr(model, "_mdl_env0")

    def hold(self):
        self.model._mdl_draw_held = None
        self.model._mdl_draw_held = next_draw_key(self.model)

    def group(self, first_env: int):
        self.model._mdl_env0 = self.env0 + int(first_env)

    def close(self):
        self.model._mdl_draw_held = None
        if self.has_env0:
            self.model._mdl_env0 = self.env0
        else:
            self.model.__dict__.pop("_mdl_env0", None)


def decode(model, rep, ava=None, deterministic=False, stride=1, rand=None):
    """rep (B, L, 64) f32 -> actions (B, L, 1), log-probs (B, L, 1)."""
    B, L, D = rep.shape
    A = model.action_dim
    pk = decoder_pack(model)
    rep = rep.float().contiguous()
    dev = rep.device
    # sampling noise: explicit draws (tests) or in-kernel Philox keyed by (model key, global env id, call counter)
    gen = rand is None and not deterministic
    rk0 = rk1 = rctr = 0
    if gen:
        rk0, rk1, rctr = next_draw_key(model)
    u = rand["u"].float().contiguous() if rand is not None else None
    n = rand["n"].float().contiguous() if rand is not None else None
    ava_c = ava.float().contiguous() if ava is not None else None
    cont, avail = pk["cont"], pk["avail"]
    out_a = torch.empty(B, L, A if cont else 1, device=dev)
    out_lp = torch.empty(B, L, (A - 1 if avail else A) if cont else 1, device=dev)
    gkey = (model.n_block, L, min(B, _EPW_CAP))
    geo = _GEO.get(gkey)
    if geo is None:
        geo = _GEO[gkey] = lib().mdl_mat_decode_geometry(*gkey)
    epw, rmax = geo & 0xFF, geo >> 8
    if epw <= 0:
        raise RuntimeError(f"mat_decode: L={L} does not fit in LDS")
    prm = DecParams(P(pk["wpack"]).value, P(pk["bias"]).value, P(pk["lnp"]).value, P(pk["emb"]).value,
                    P(pk["wh2"]).value, P(pk["bh2"]).value, P(pk["stdv"]).value, P(rep).value, P(ava_c).value,
                    P(u).value, P(n).value, P(out_a).value, P(out_lp).value,
                    B, L, A, _n_disc(model, L), int(stride if deterministic else 1), int(bool(deterministic)), epw, rmax,
                    pk["n_tok"], pk["tok_start"], pk["tok_zero"], 0, cont,
                    P(pk.get("wa")).value, P(pk.get("ba")).value, P(pk.get("lnd")).value, int(gen), rk0, rk1, rctr,
                    avail, P(pk.get("qkv0")).value, 0, int(getattr(model, "_mdl_env0", 0)) & 0xFFFFFFFF,
                    P(pk.get("hfold")).value, P(pk.get("wfa") if WAVE_DECODE else None).value)
    if _spec_set[0] != SPEC_DECODE:
        lib().mdl_decode_spec_enable(int(SPEC_DECODE))
        _spec_set[0] = SPEC_DECODE
    # the path report (two plan queries + formatting) once per call shape, not per rollout step
    pkey = (B, L, A, model.n_block, int(bool(deterministic)), int(stride), cont, avail, gen, rand is not None,
            ava is not None, WAVE_DECODE, SPEC_DECODE, id(pk))
    if getattr(model, "_mdl_decode_path_key", None) != pkey:
        model._mdl_decode_path = wave_path(prm, model.n_block)
        model._mdl_decode_path_key = pkey
    check(lib().mdl_mat_decode(ctypes.byref(prm), model.n_block, kernels._stream()), "mat_decode")
    return out_a, out_lp


_GEO = {}   # mdl_mat_decode_geometry results (a pure function of its arguments)


def wave_path(prm, n_block):
    """'spec(nreg=k)' when the decode call runs on the speculative-block-0 kernel (k main-wave matrices
    register-resident), 'wave(nreg=k)' on the one-wave kernel, else '4wave'."""
    k = lib().mdl_decode_spec_plan(ctypes.byref(prm), n_block)
    if k >= 0:
        return f"spec(nreg={k & 15}{', tokrows' if k & 16 else ''}{', q2inline' if k & 32 else ''})"
    k = lib().mdl_decode_wave_plan(ctypes.byref(prm), n_block)
    return f"wave(nreg={k})" if k >= 0 else "4wave"


def _encode(model, obs):
    from . import mat_train
    if mat_train.encoder_supported(model):
        return mat_train.encode(model, obs)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        v, rep = model.encoder(None, obs)
    return v.float(), rep.float()


@torch.no_grad()
def get_actions(model, obs, ava=None, deterministic=False, stride=1, rand=None):
    v, rep = _encode(model, obs)
    a, lp = decode(model, rep, ava, deterministic, stride, rand)
    return v, a, lp


@torch.no_grad()
def get_values_rep(model, obs):
    """(values, rep) from the fused encoder (eager fallback when its gates reject the model)."""
    return _encode(model, obs)


@torch.no_grad()
def get_values(model, obs):
    return _encode(model, obs)[0]


def evaluate_actions(model, obs, actions, ava=None):
    from . import mat_train
    if mat_train.supported(model):
        return mat_train.evaluate_actions(model, obs, actions, ava)
    from ..models import act as act_mod
    if mat_train.encoder_supported(model) and not model.encoder.encode_state:
        # hybrid: fused encoder fwd/bwd kernels, eager decoder (its gates rejected the model)
        v, rep = mat_train.encode_train(model, obs)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logp, ent = act_mod.parallel_act(model, rep, obs, actions, ava)
        return v, logp.float(), ent.float()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        v, rep = model.encoder(None, obs)
        logp, ent = act_mod.parallel_act(model, rep, obs, actions, ava)
    return v.float(), logp, ent
