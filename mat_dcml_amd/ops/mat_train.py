"""Bindings of the fused MAT kernels: training forward/backward (``csrc/mat_train.hip``) and the weight packs.

* ``ModelPack`` — every 64x64 Linear of the MAT in MFMA B-fragment order, for W (forward) and Wᵀ (backward), in
  two persistent bf16 buffers.  One ``pack_weights`` launch refreshes all of them after an optimizer step
  (tracked by ``model._mdl_version``).  Biases / LayerNorm parameters are read in place (fp32).
* ``EncoderFused`` / ``DecoderFused`` — the whole-encoder / whole-decoder (teacher-forced) forward with the
  activations the backward needs, and the backward, which writes parameter gradients straight into ``.grad``
  (fp32 atomics; the grads are views of one flat buffer, see ``parallel/comm.FlatGrads``).
* ``evaluate_actions`` — autograd entry used by the PPO trainer: (values, log-probs, entropy) of stored actions.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import kernels
from .kernels import P, check, lib, sig
from .ppo_fused import AdamArgs

VP = ctypes.c_void_p


class Mat(ctypes.Structure):
    _fields_ = [("fw", VP), ("bw", VP), ("b", VP), ("dW", VP), ("db", VP), ("fa", VP), ("ba", VP)]


class LNp(ctypes.Structure):
    _fields_ = [("g", VP), ("b", VP), ("dg", VP), ("db", VP)]


class Blk(ctypes.Structure):
    _fields_ = [("m", Mat * 10), ("ln", LNp * 3)]


class Sv(ctypes.Structure):
    # g / gp: the MLP's GELU(h) and GELU'(h) as bf16 (the backward recomputes neither); xh0..2 / rs: x-hat (bf16) and
    # rstd ([tok][4] f32) of the block's LayerNorms (the backward recomputes no LayerNorm forward)
    _fields_ = [(n, VP) for n in ("xin", "a1", "lse1", "x1", "a2", "lse2", "x2", "g", "a1lo", "a2lo", "gp", "xh0", "xh1",
                                  "xh2", "rs")]


class HSv(ctypes.Structure):
    # x-hat, GELU'(pre-activation) (bf16 [tok][64]) and rstd ([tok] f32) of a GELU -> LayerNorm head / embedding
    _fields_ = [("xh", VP), ("gp", VP), ("rs", VP)]


class EncP(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("Bs", "L", "od", "SQ", "NRP", "n_obj")] + \
               [(n, VP) for n in ("obs", "lno_g", "lno_b", "we", "be", "ln0_g", "ln0_b", "d_lno_g", "d_lno_b", "d_we",
                                  "d_be", "d_ln0_g", "d_ln0_b")] + \
               [("blk", Blk * 3), ("h1", Mat), ("lnh", LNp), ("wh2", VP), ("bh2", VP), ("d_wh2", VP), ("rep", VP),
                ("v", VP), ("sv", Sv * 3), ("drep", VP), ("dv", VP), ("g_delta", ctypes.c_longlong),
                ("g_stride", ctypes.c_longlong), ("g_copies", ctypes.c_int), ("d_bh2", VP), ("hs", HSv), ("es", HSv),
                ("g_mode", ctypes.c_int), ("sidx", VP)]


class DecP(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("Bs", "L", "A", "SQ", "NRP", "n_disc")] + \
               [(n, VP) for n in ("act", "ava", "wa", "d_wa", "lnd_g", "lnd_b", "d_lnd_g", "d_lnd_b")] + \
               [("blk", Blk * 3), ("h1", Mat), ("lnh", LNp)] + \
               [(n, VP) for n in ("wh2", "bh2", "d_wh2", "d_bh2", "stdv", "log_std", "d_log_std", "rep", "logp",
                                  "ent")] + \
               [("sv", Sv * 3)] + [(n, VP) for n in ("dlogp", "dent", "drep", "sv_head")] + \
               [("g_delta", ctypes.c_longlong), ("g_stride", ctypes.c_longlong), ("g_copies", ctypes.c_int)] + \
               [("cont", ctypes.c_int), ("ba", VP), ("d_ba", VP), ("hs", HSv), ("g_mode", ctypes.c_int), ("sidx", VP)]


# Training kernels (csrc/mat_train_ct.h): token-on-lane tiles, weight A fragments in permuted k order, register-
# chained linears.  The forward kernels run 4 waves x 2 workgroups per CU, the backward 8 waves x 1 (its own
# translation units); the tile geometry comes from mdl_mat_train_geometry_ct.
sig("mdl_mat_train_geometry_ct", ctypes.c_int)
sig("mdl_mat_enc_fwd_ct", ctypes.POINTER(EncP), VP, ctypes.c_int, ctypes.c_int, VP)
sig("mdl_mat_enc_bwd_ct", ctypes.POINTER(EncP), VP, VP, ctypes.c_int, VP)
sig("mdl_mat_dec_fwd_ct", ctypes.POINTER(DecP), ctypes.c_int, ctypes.c_int, VP)
sig("mdl_mat_dec_bwd_ct", ctypes.POINTER(DecP), ctypes.c_int, VP)
sig("mdl_grad_reduce", VP, VP, ctypes.c_int, ctypes.c_longlong, ctypes.c_int, VP)
sig("mdl_grad_reduce_norm", VP, VP, ctypes.c_int, ctypes.c_longlong, ctypes.c_int, VP, VP)
sig("mdl_grad_reduce_priv", VP, VP, VP, ctypes.c_int, ctypes.c_int, ctypes.c_longlong, ctypes.c_int, ctypes.c_int, VP, VP)
sig("mdl_ct_bwd_grid", ctypes.c_int, ctypes.c_int)


class OEArgs(ctypes.Structure):   # csrc/obs_embed.hip
    _fields_ = [(n, ctypes.c_int) for n in ("N", "od", "KS")] + \
               [(n, VP) for n in ("x", "we", "be", "g", "b", "wpack", "c01", "pre", "stat", "dpre", "M", "ud", "d_we",
                                  "d_be", "d_g", "d_b", "xh")]


sig("mdl_obs_embed_pack", ctypes.POINTER(OEArgs), VP)
sig("mdl_obs_embed_fwd", ctypes.POINTER(OEArgs), VP)
sig("mdl_obs_embed_bwd", ctypes.POINTER(OEArgs), VP)
MAX_FUSED_OBS = 16      # obs_dim embedded inside the fused encoder; wider observations use csrc/obs_embed.hip
# Wide observations (SMAC's 1,288 features) enter the embedding as bf16: half the bytes of its one large operand.
# Rollout and learner both round them, so the PPO ratio is unaffected (tests/test_gpu_logprob_consistency.py smac).
# SMAC bench 75.8k / 76.8k -> 77.8k / 77.8k env-steps/s (profiles/r6_ab/).  MAT_DCML_WIDE_OBS_BF16=0: fp32 inputs.
WIDE_OBS_BF16 = os.environ.get("MAT_DCML_WIDE_OBS_BF16", "1") == "1"


class ObsEmbed:
    """LN(obs_dim) -> Linear(obs_dim, 64) pre-activation on MFMA for wide observations (SMAC), with the LayerNorm
    folded into the GEMM (csrc/obs_embed.hip); its W' pack is refreshed once per optimizer step."""

    def __init__(self, model):
        enc = model.encoder
        self.model = model
        self.ln, self.lin = enc.obs_encoder[0], enc.obs_encoder[1]
        self.od = enc.obs_dim
        self.KS = (self.od + 31) // 32
        dev = self.lin.weight.device
        self.wpack = torch.empty(self.KS * 4 * 64 * 8, dtype=torch.bfloat16, device=dev)
        self.c01 = torch.empty(128, device=dev)
        self.M = torch.empty(64 * self.od, device=dev)
        self.ud = torch.empty(128, device=dev)
        self.version = None

    def _args(self, N=0, x=None, pre=None, stat=None, dpre=None):
        xh = x if x is not None and x.dtype == torch.bfloat16 else None
        if xh is not None:
            x = None
        return OEArgs(N=N, od=self.od, KS=self.KS, x=_ptr(x), xh=_ptr(xh), we=self.lin.weight.data_ptr(),
                      be=self.lin.bias.data_ptr(),
                      g=self.ln.weight.data_ptr(), b=self.ln.bias.data_ptr(), wpack=self.wpack.data_ptr(),
                      c01=self.c01.data_ptr(), pre=_ptr(pre), stat=_ptr(stat), dpre=_ptr(dpre), M=self.M.data_ptr(),
                      ud=self.ud.data_ptr(), d_we=_gptr(self.lin.weight), d_be=_gptr(self.lin.bias),
                      d_g=_gptr(self.ln.weight), d_b=_gptr(self.ln.bias))

    def refresh(self):
        ver = getattr(self.model, "_mdl_version", 0)
        if ver != self.version:
            a = self._args()
            check(lib().mdl_obs_embed_pack(ctypes.byref(a), kernels._stream()), "obs_embed_pack")
            self.version = ver

    def forward(self, obs2d):
        self.refresh()
        N = obs2d.shape[0]
        pre = torch.empty(N, 64, device=obs2d.device)
        stat = torch.empty(N, 2, device=obs2d.device)
        a = self._args(N, obs2d, pre, stat)
        check(lib().mdl_obs_embed_fwd(ctypes.byref(a), kernels._stream()), "obs_embed_fwd")
        return pre, stat

    def backward(self, obs2d, stat, dpre):
        a = self._args(obs2d.shape[0], obs2d, None, stat, dpre)
        check(lib().mdl_obs_embed_bwd(ctypes.byref(a), kernels._stream()), "obs_embed_bwd")
sig("mdl_pack_weights", VP, ctypes.c_int, VP)

MAX_ACTION_DIM = 64


def _spread(B, L, SQ, NRP, dev):
    """Fewer sequences per workgroup when B / SQ tiles would leave CUs idle (the rollout encoder at 256 envs ran
    52 workgroups of 5 sequences on a 256-CU device)."""
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count if dev.type == "cuda" else 1
    sq = max(1, min(SQ, -(-B // n_cu)))
    if sq == SQ:
        return SQ, NRP
    return sq, max(64, ((sq * L + 31) // 32) * 32)


def geometry(L):
    """(SQ sequences per tile, NRP padded rows, kernel suffix) of the training tiling for sequence length L
    ((0, 0, "") when L does not fit)."""
    v = lib().mdl_mat_train_geometry_ct(L)
    return (v & 0xFFFF, v >> 16, "_ct") if v else (0, 0, "")


def _enc_fwd(sfx, p, pre_in, nb, save):
    return lib().mdl_mat_enc_fwd_ct(ctypes.byref(p), pre_in, nb, int(save), kernels._stream())


def _enc_bwd(sfx, p, pre_in, dpre_out, nb):
    return lib().mdl_mat_enc_bwd_ct(ctypes.byref(p), pre_in, dpre_out, nb, kernels._stream())


def _ptr(t):
    return t.data_ptr() if t is not None else None


def _gptr(t):
    return t.grad.data_ptr() if t.grad is not None else None


# ------------------------------------------------------------------------------------------------- packs
def decoder_linears(model):
    dec = model.decoder
    out = []
    if dec.dec_actor:   # MAT-Dec: per-agent MLP actors, no transformer blocks to pack (hybrid path: eager decoder)
        return out
    for blk in dec.blocks:
        a1, a2 = blk.attn1, blk.attn2
        out += [a1.query, a1.key, a1.value, a1.proj, a2.query, a2.key, a2.value, a2.proj, blk.mlp[0], blk.mlp[2]]
    out.append(dec.head[0])
    return out


def encoder_linears(model):
    enc = model.encoder
    out = []
    for blk in enc.blocks:
        a = blk.attn
        out += [a.query, a.key, a.value, a.proj, blk.mlp[0], blk.mlp[2]]
    out.append(enc.head[0])
    return out


class ModelPack:
    def __init__(self, model):
        self.model = model
        lins = decoder_linears(model) + encoder_linears(model)
        self.n = len(lins)
        self.n_dec = len(decoder_linears(model))
        dev = lins[0].weight.device
        self.fw = torch.empty(self.n, 4096, dtype=torch.bfloat16, device=dev)
        self.fa = torch.empty(self.n, 4096, dtype=torch.bfloat16, device=dev)
        self.ba = torch.empty(self.n, 4096, dtype=torch.bfloat16, device=dev)
        self.index = {id(l): i for i, l in enumerate(lins)}
        tab = [[l.weight.data_ptr(), self.fw[i].data_ptr(), 0, self.fa[i].data_ptr(),
                self.ba[i].data_ptr()] for i, l in enumerate(lins)]
        self.table = torch.tensor(tab, dtype=torch.int64, device=dev)
        self.version = None

    def refresh(self):
        ver = getattr(self.model, "_mdl_version", 0)
        if ver != self.version:
            check(lib().mdl_pack_weights(P(self.table), self.n, kernels._stream()), "pack_weights")
            self.version = ver

    def mat(self, lin):
        i = self.index[id(lin)]
        return Mat(self.fw[i].data_ptr(), None, lin.bias.data_ptr(), _gptr(lin.weight),
                   _gptr(lin.bias), self.fa[i].data_ptr(), self.ba[i].data_ptr())

    @property
    def decoder_fw(self):
        return self.fw[: self.n_dec]


def model_pack(model):
    mp = getattr(model, "_mdl_pack", None)
    if mp is None:
        mp = ModelPack(model)
        model._mdl_pack = mp
    mp.refresh()
    return mp


def _ln(ln):
    return LNp(ln.weight.data_ptr(), ln.bias.data_ptr(), _gptr(ln.weight), _gptr(ln.bias))


def _grad_sig(model):
    """Gradient-pointer signature the packed kernel arguments were built against: the first encoder AND decoder
    parameter (the hybrid path creates encoder gradients separately from the decoder's autograd ones)."""
    ps = (next(model.encoder.parameters()), next(model.decoder.parameters()))
    return tuple(p.grad.data_ptr() if p.grad is not None else 0 for p in ps)


# ------------------------------------------------------------------------------------------------- support
def _common_reasons(model):
    if not kernels.available():
        return ["HIP library not loaded (kernels=torch or not built)"]
    r = []
    if model.n_embd != 64 or model.n_head != 2 or model.n_block not in (1, 2, 3):
        r.append(f"n_embd {model.n_embd} / n_head {model.n_head} / n_block {model.n_block} (kernel: 64 / 2 / 1-3)")
    if geometry(model.n_agent)[0] <= 0:
        r.append(f"L={model.n_agent} does not fit the training tiling")
    return r


def encoder_unsupported_reasons(model):
    enc = model.encoder
    r = _common_reasons(model)
    if enc.encode_state:
        r.append("encode_state")
    if model.n_objective > 2:
        r.append(f"n_objective {model.n_objective} > 2")
    return r


def decoder_unsupported_reasons(model):
    dec = model.decoder
    r = _common_reasons(model)
    if dec.dec_actor:
        r.append("dec_actor")
    ok_types = ("Semi_Discrete", "Discrete", "Continuous", "Continous")
    if model.action_type not in ok_types:
        r.append(f"action_type {model.action_type}")
    if model.action_dim > MAX_ACTION_DIM:
        r.append(f"action_dim {model.action_dim} > {MAX_ACTION_DIM}")
    if model.action_type == "Semi_Discrete" and model.semi_index != -1:
        r.append(f"semi_index {model.semi_index} != -1")
    return r


def encoder_supported(model):
    return not encoder_unsupported_reasons(model)


def decoder_supported(model):
    return not decoder_unsupported_reasons(model)


def supported(model):
    return encoder_supported(model) and decoder_supported(model)


# ------------------------------------------------------------------------------------------------- encoder
class EncoderFused:
    def __init__(self, model):
        self.model = model
        self.p = None
        self.sig = None

    def _build(self):
        m = self.model
        s = _grad_sig(m)
        if self.p is not None and self.sig == s:
            return
        mp = model_pack(m)
        enc = m.encoder
        p = EncP()
        ln_o, lin_e = enc.obs_encoder[0], enc.obs_encoder[1]
        for name, t in (("lno_g", ln_o.weight), ("lno_b", ln_o.bias), ("we", lin_e.weight), ("be", lin_e.bias),
                        ("ln0_g", enc.ln.weight), ("ln0_b", enc.ln.bias)):
            setattr(p, name, t.data_ptr())
            setattr(p, "d_" + name, _gptr(t))
        for bi, blk in enumerate(enc.blocks):
            a = blk.attn
            for slot, lin in ((0, a.query), (1, a.key), (2, a.value), (3, a.proj), (8, blk.mlp[0]), (9, blk.mlp[2])):
                p.blk[bi].m[slot] = mp.mat(lin)
            p.blk[bi].ln[0] = _ln(blk.ln1)
            p.blk[bi].ln[1] = _ln(blk.ln2)
        p.h1 = mp.mat(enc.head[0])
        p.lnh = _ln(enc.head[2])
        p.wh2, p.bh2, p.d_wh2 = enc.head[3].weight.data_ptr(), enc.head[3].bias.data_ptr(), _gptr(enc.head[3].weight)
        self.p, self.sig = p, s

    def refresh_packs(self):
        """Build every version-keyed weight pack the forward reads (shared ModelPack, the wide-observation embedding
        pack) on the CURRENT stream — see mat_fused.refresh_packs."""
        model_pack(self.model)
        if self.model.encoder.obs_dim > MAX_FUSED_OBS:
            if getattr(self, "emb", None) is None:
                self.emb = ObsEmbed(self.model)
            self.emb.refresh()

    def forward(self, obs, save=True, idx=None):
        """obs (B, L, od) -> (v (B, L, n_obj), rep (B, L, 64) f32).  ``idx`` (int64 [B]): obs is the rollout
        buffer (N, L, od) and minibatch sequence s reads its row idx[s] in-kernel (no gather copy)."""
        m = self.model
        model_pack(m)
        self._build()
        _, L, od = obs.shape
        B = obs.shape[0] if idx is None else idx.numel()
        dev = obs.device
        SQ, NRP, sfx = geometry(L)
        if not save:   # rollout / value passes: small batches — spread them over every CU (nothing is saved, so
            SQ, NRP = _spread(B, L, SQ, NRP, dev)   # the backward's tiling need not match)
        n_tok = B * L
        wide_bf16 = od > MAX_FUSED_OBS and (WIDE_OBS_BF16 or obs.dtype == torch.bfloat16)
        obs = (obs.to(torch.bfloat16) if wide_bf16 else obs.float()).contiguous()
        pre = stat = None
        if od > MAX_FUSED_OBS:   # wide observations: embedding pre-activation from the obs-embedding kernel
            if idx is not None:  # (the wide embedding reads dense rows)
                obs, idx = obs[idx].contiguous(), None
            if getattr(self, "emb", None) is None:
                self.emb = ObsEmbed(m)
            pre, stat = self.emb.forward(obs.view(n_tok, od))
        rep = torch.empty(B, L, 64, device=dev)
        v = torch.empty(B, L, m.n_objective, device=dev)
        p = self.p
        p.Bs, p.L, p.od, p.SQ, p.NRP, p.n_obj = B, L, od, SQ, NRP, m.n_objective
        p.obs, p.rep, p.v, p.sidx = obs.data_ptr(), rep.data_ptr(), v.data_ptr(), _ptr(idx)
        saves = []
        if save:
            for bi in range(m.n_block):
                t = torch.empty(8, n_tok, 64, device=dev, dtype=torch.bfloat16)
                lse = torch.empty(n_tok, 2, device=dev)
                rs = torch.empty(3, n_tok, device=dev)   # LayerNorm rstd, slot-major
                saves += [t, lse, rs]
                p.sv[bi] = Sv(t[0].data_ptr(), t[1].data_ptr(), lse.data_ptr(), t[2].data_ptr(), None, None, None,
                              t[3].data_ptr(), t[4].data_ptr(), None, t[5].data_ptr(), t[6].data_ptr(), t[7].data_ptr(),
                              None, rs.data_ptr())
            hv = torch.empty(4, n_tok, 64, device=dev, dtype=torch.bfloat16)   # head / embedding x-hat, GELU'
            hr = torch.empty(2, n_tok, device=dev)                              # head / embedding rstd
            saves += [hv, hr]
            p.hs = HSv(hv[0].data_ptr(), hv[1].data_ptr(), hr[0].data_ptr())
            p.es = HSv(hv[2].data_ptr(), hv[3].data_ptr(), hr[1].data_ptr())
        else:
            p.hs, p.es = HSv(), HSv()
        check(_enc_fwd(sfx, p, _ptr(pre), m.n_block, save), "mat_enc_fwd")
        self.ctx = (obs, rep, v, saves, [Sv.from_buffer_copy(p.sv[i]) for i in range(m.n_block)], pre, stat,
                    HSv.from_buffer_copy(p.hs), HSv.from_buffer_copy(p.es), idx)
        return v, rep

    def backward(self, drep, dv):
        m = self.model
        obs, rep, v, saves, svs, pre, stat, hs, es, idx = self.ctx
        self._build()
        p = self.p
        p.hs, p.es = hs, es
        drep = drep.float().contiguous()
        dv = dv.float().contiguous()
        B, L, od = rep.shape[0], obs.shape[1], obs.shape[2]
        SQ, NRP, sfx = geometry(L)
        p.Bs, p.L, p.od, p.SQ, p.NRP, p.n_obj = B, L, od, SQ, NRP, m.n_objective
        p.obs, p.rep, p.v, p.drep, p.dv = obs.data_ptr(), rep.data_ptr(), v.data_ptr(), drep.data_ptr(), dv.data_ptr()
        p.sidx = _ptr(idx)
        for i, s in enumerate(svs):
            p.sv[i] = s
        _set_workspace(p, m, B, SQ)
        dpre = torch.empty_like(pre) if pre is not None else None
        b = m.encoder.head[3].bias
        in_kernel = b.grad is not None   # the backward kernel sums dv into the bias gradient itself
        p.d_bh2 = b.grad.data_ptr() if in_kernel else None
        if in_kernel and p.g_copies:
            check_grad_ptrs(p, m._mdl_gws_buf[1])
        check(_enc_bwd(sfx, p, _ptr(pre), _ptr(dpre), m.n_block), "mat_enc_bwd")
        if pre is not None:
            self.emb.backward(obs.view(-1, od), stat, dpre)
        if b.grad is not None and not in_kernel:
            b.grad.add_(dv.reshape(-1, dv.shape[-1]).sum(0))


# ------------------------------------------------------------------------------------------------- decoder
class DecoderFused:
    def __init__(self, model):
        self.model = model
        self.p = None
        self.sig = None

    def _build(self):
        m = self.model
        s = _grad_sig(m)
        if self.p is not None and self.sig == s:
            return
        mp = model_pack(m)
        dec = m.decoder
        p = DecP()
        p.wa, p.d_wa = dec.action_encoder[0].weight.data_ptr(), _gptr(dec.action_encoder[0].weight)
        self.cont = m.action_type in ("Continuous", "Continous")
        if self.cont:   # Linear(A, 64) with bias on the previous agent's action vector
            p.cont, p.ba, p.d_ba = 1, dec.action_encoder[0].bias.data_ptr(), _gptr(dec.action_encoder[0].bias)
        p.lnd_g, p.lnd_b, p.d_lnd_g, p.d_lnd_b = dec.ln.weight.data_ptr(), dec.ln.bias.data_ptr(), \
            _gptr(dec.ln.weight), _gptr(dec.ln.bias)
        for bi, blk in enumerate(dec.blocks):
            a1, a2 = blk.attn1, blk.attn2
            for slot, lin in ((0, a1.query), (1, a1.key), (2, a1.value), (3, a1.proj), (4, a2.query), (5, a2.key),
                              (6, a2.value), (7, a2.proj), (8, blk.mlp[0]), (9, blk.mlp[2])):
                p.blk[bi].m[slot] = mp.mat(lin)
            p.blk[bi].ln[0] = _ln(blk.ln1)
            p.blk[bi].ln[1] = _ln(blk.ln2)
            p.blk[bi].ln[2] = _ln(blk.ln3)
        p.h1 = mp.mat(dec.head[0])
        p.lnh = _ln(dec.head[2])
        h3 = dec.head[3]
        p.wh2, p.bh2, p.d_wh2, p.d_bh2 = h3.weight.data_ptr(), h3.bias.data_ptr(), _gptr(h3.weight), _gptr(h3.bias)
        if m.action_type != "Discrete":
            self.std = torch.empty(m.action_dim, device=h3.weight.device)
            p.log_std, p.stdv, p.d_log_std = dec.log_std.data_ptr(), self.std.data_ptr(), _gptr(dec.log_std)
        else:
            self.std = torch.ones(m.action_dim, device=h3.weight.device)
            p.log_std, p.stdv, p.d_log_std = self.std.data_ptr(), self.std.data_ptr(), None
        self.p, self.sig = p, s

    def _n_disc(self, L):
        m = self.model
        if m.action_type == "Discrete":
            return L
        if m.action_type in ("Continuous", "Continous"):
            return 0
        return L + m.semi_index

    def _geom(self, B, L):
        SQ, NRP, sfx = geometry(L)
        p = self.p
        p.Bs, p.L, p.A, p.SQ, p.NRP, p.n_disc = B, L, self.model.action_dim, SQ, NRP, self._n_disc(L)
        return sfx

    def forward(self, rep, actions, ava=None, save=True, idx=None):
        """``idx`` (int64 [B]): actions / ava are the rollout buffer's (N, L, .) rows, read through idx in-kernel."""
        m = self.model
        model_pack(m)
        self._build()
        B, L, _ = rep.shape
        dev = rep.device
        n_tok = B * L
        rep = rep.float().contiguous()
        nlp = m.action_dim if self.cont else 1   # continuous: per-dimension actions / log-probs / entropies
        nrow = B if idx is None else actions.shape[0]
        act = actions.reshape(nrow, L, nlp).float().contiguous()
        ava_c = ava.float().contiguous() if (ava is not None and not self.cont) else None
        logp = torch.empty(B, L, nlp, device=dev)
        ent = torch.empty(B, L, nlp, device=dev)
        sfx = self._geom(B, L)
        p = self.p
        p.act, p.ava, p.rep, p.logp, p.ent = act.data_ptr(), _ptr(ava_c), rep.data_ptr(), logp.data_ptr(), ent.data_ptr()
        p.sidx = _ptr(idx)
        saves = []
        if save:
            for bi in range(m.n_block):
                t = torch.empty(12, n_tok, 64, device=dev, dtype=torch.bfloat16)
                lse = torch.empty(2, n_tok, 2, device=dev)
                rs = torch.empty(3, n_tok, device=dev)   # LayerNorm rstd, slot-major
                saves += [t, lse, rs]
                p.sv[bi] = Sv(t[0].data_ptr(), t[1].data_ptr(), lse[0].data_ptr(), t[2].data_ptr(), t[3].data_ptr(),
                              lse[1].data_ptr(), t[4].data_ptr(), t[5].data_ptr(), t[6].data_ptr(), t[7].data_ptr(),
                              t[8].data_ptr(), t[9].data_ptr(), t[10].data_ptr(), t[11].data_ptr(), rs.data_ptr())
            head = torch.empty(3, n_tok, 64, device=dev, dtype=torch.bfloat16)   # head input, x-hat, GELU'
            hr = torch.empty(n_tok, device=dev)
            saves += [head, hr]
            p.sv_head = head[0].data_ptr()
            p.hs = HSv(head[1].data_ptr(), head[2].data_ptr(), hr.data_ptr())
        else:
            p.hs = HSv()
        check(getattr(lib(), "mdl_mat_dec_fwd" + sfx)(ctypes.byref(p), m.n_block, int(save), kernels._stream()), "mat_dec_fwd")
        self.ctx = (rep, act, ava_c, logp, ent, saves, [Sv.from_buffer_copy(p.sv[i]) for i in range(m.n_block)],
                    p.sv_head, HSv.from_buffer_copy(p.hs), idx)
        return logp, ent

    def backward(self, dlogp, dent):
        m = self.model
        rep, act, ava_c, logp, ent, saves, svs, head, hs, idx = self.ctx
        self._build()
        B, L = rep.shape[:2]
        sfx = self._geom(B, L)
        p = self.p
        dlogp = dlogp.reshape(-1).float().contiguous()
        dent = dent.reshape(-1).float().contiguous()
        # the backward writes every row of d rep (its last decoder block overwrites)
        drep = torch.empty_like(rep)
        p.act, p.ava, p.rep, p.sidx = act.data_ptr(), _ptr(ava_c), rep.data_ptr(), _ptr(idx)
        p.dlogp, p.dent, p.drep, p.sv_head = dlogp.data_ptr(), dent.data_ptr(), drep.data_ptr(), head
        p.hs = hs
        for i, s in enumerate(svs):
            p.sv[i] = s
        _set_workspace(p, m, B, p.SQ)
        check(getattr(lib(), "mdl_mat_dec_bwd" + sfx)(ctypes.byref(p), m.n_block, kernels._stream()), "mat_dec_bwd")
        return drep


class _MATFusedFn(torch.autograd.Function):
    """(anchor, obs, actions, ava) -> (logp, values, entropy); backward runs the fused decoder then encoder
    backward kernels, which write the parameter gradients straight into ``.grad``."""

    @staticmethod
    def forward(ctx, anchor, obs, actions, ava, enc, dec):
        v, rep = enc.forward(obs, save=True)
        logp, ent = dec.forward(rep, actions, ava, save=True)
        # the saved activations belong to THIS forward: another fused call before backward (a second
        # evaluate_actions, get_values) overwrites enc.ctx / dec.ctx, so they are restored from here
        ctx.enc, ctx.dec, ctx.saved = enc, dec, (enc.ctx, dec.ctx)
        return logp, v, ent

    @staticmethod
    def backward(ctx, dlogp, dv, dent):
        dec, enc = ctx.dec, ctx.enc
        enc.ctx, dec.ctx = ctx.saved
        ctx.saved = None
        logp, ent = dec.ctx[3], dec.ctx[4]
        drep = dec.backward(dlogp if dlogp is not None else torch.zeros_like(logp),
                            dent if dent is not None else torch.zeros_like(ent))
        enc.backward(drep, dv if dv is not None else torch.zeros_like(enc.ctx[2]))
        dec.ctx = None
        enc.ctx = None
        return torch.zeros((), device=drep.device), None, None, None, None, None


GRAD_MODES = ("private", "atomic")


def attach_grad_workspace(model, flat_grads: torch.Tensor, copies: int = 32, mode: str = "atomic"):
    """Gradient workspace of the backward kernels (every parameter's ``.grad`` must be a view of ``flat_grads``);
    ``reduce_grad_workspace`` folds it back.
    * ``atomic`` (rounds 2-5): the weight-gradient fp32 atomics spread over ``copies`` shared copies (fewer
      workgroups adding into one 16 KB matrix);
    * ``private`` (round 6, the trainer's default): ONE copy per workgroup of the persistent backward launches
      (``copies`` is raised to the device's CU count), written with plain stores / read-modify-writes — no atomics,
      a fixed summation order, a bit-reproducible gradient (csrc/mat_train_common.h GradMode).  The 64 x 64 weight
      gradients sit in the copies in MFMA fragment order; ``dst`` maps them back."""
    assert mode in GRAD_MODES, mode
    n = flat_grads.numel()
    if mode == "private":
        copies = max(copies, int(lib().mdl_ct_bwd_grid(1 << 30, 1)))   # = n_cus(): the largest backward grid
    stride = (n + 63) // 64 * 64
    ws = torch.zeros(copies * stride, dtype=torch.float32, device=flat_grads.device)
    delta = (ws.data_ptr() - flat_grads.data_ptr()) // 4
    assert (ws.data_ptr() - flat_grads.data_ptr()) % 4 == 0
    model._mdl_gws = (delta, stride, copies)
    model._mdl_gws_buf = (ws, flat_grads, stride, copies)
    model._mdl_gws_mode = mode
    model._mdl_gws_grid = None
    if mode == "private":
        model._mdl_gws_dst = _fragment_dst(model, flat_grads)
    return ws


def _fragment_dst(model, flat):
    """int32 [n]: where element s of a private workspace copy goes in the flat gradient.  Identity, except inside the
    64 x 64 weight gradients the kernels flush in fragment order (wgrad64 / wgrad64_shared_x: every ModelPack linear):
    s = o + wave * 512 + lane * 8 + 4 j + r  ->  o + 64 (16 (wave & 3) + 4 (lane >> 4) + r) + 16 (2 (wave >> 2) + j)
    + (lane & 15)."""
    n = flat.numel()
    dst = torch.arange(n, dtype=torch.int64)
    f = torch.arange(4096)
    wave, lane, j, r = f >> 9, (f >> 3) & 63, (f >> 2) & 1, f & 3
    row = 16 * (wave & 3) + 4 * (lane >> 4) + r
    col = 16 * (2 * (wave >> 2) + j) + (lane & 15)
    perm = row * 64 + col
    assert torch.equal(perm.sort().values, f)
    for lin in decoder_linears(model) + encoder_linears(model):
        g = lin.weight.grad
        if g is None or g.numel() != 4096:
            continue
        o = (g.data_ptr() - flat.data_ptr()) // 4
        assert 0 <= o and o + 4096 <= n
        dst[o:o + 4096] = o + perm
    return dst.to(torch.int32).to(flat.device)


def _set_workspace(p, m, B, SQ):
    """Point the backward's gradient fields at the model's workspace (when the trainer activated it)."""
    if getattr(m, "_mdl_gws_active", False):
        p.g_delta, p.g_stride, p.g_copies = m._mdl_gws
        p.g_mode = int(getattr(m, "_mdl_gws_mode", "atomic") == "private")
        check_grad_ptrs(p, m._mdl_gws_buf[1])
        if p.g_mode:
            grid = int(lib().mdl_ct_bwd_grid(B, SQ))
            if m._mdl_gws_grid not in (None, grid):
                raise RuntimeError(f"private gradient workspace: backward grids {m._mdl_gws_grid} and {grid} differ "
                                   "within one minibatch")
            m._mdl_gws_grid = grid
    else:
        p.g_delta, p.g_stride, p.g_copies, p.g_mode = 0, 0, 0, 0


def _grad_ptr_fields(st, prefix=""):
    """All gradient pointers of an EncP / DecP ctypes struct (d_* / dW / db / dg / db fields), recursively."""
    out = []
    for name, typ in st._fields_:
        v = getattr(st, name)
        if isinstance(v, ctypes.Array):
            for i, e in enumerate(v):
                if isinstance(e, ctypes.Structure):
                    out += _grad_ptr_fields(e, f"{prefix}{name}[{i}].")
        elif isinstance(v, ctypes.Structure):
            out += _grad_ptr_fields(v, f"{prefix}{name}.")
        elif (name.startswith("d_") or name in ("dW", "db", "dg")) and v:
            out.append((prefix + name, v))
    return out


def check_grad_ptrs(p, flat):
    """Host-side guard for the gradient workspace: every gradient pointer must lie inside ``flat``."""
    lo, hi = flat.data_ptr(), flat.data_ptr() + flat.numel() * 4
    bad = [(n, v) for n, v in _grad_ptr_fields(p) if not (lo <= v < hi)]
    if bad:
        raise RuntimeError(f"gradient pointers outside the flat gradient buffer: {bad[:6]} (flat {lo:#x}..{hi:#x})")


def reduce_grad_workspace(model, lo=0, hi=None, norm_into=None, accumulate=True, last=True):
    """Fold the workspace copies of flat-gradient elements [lo, hi) back into the flat buffer.
    ``norm_into`` (the whole buffer only): also write the optimizer's Σ g² partials of the final gradient into that
    FlatAdam scratch (``FlatAdam.step(norm_ready=True)`` then skips its norm launch).  Returns whether it did.
    Atomic copies are added to the buffer and zeroed; private copies are summed in copy order over the workgroups of
    the minibatch's backward launches, and ``accumulate=False`` overwrites the buffer (no zero fill needed when
    nothing else wrote gradients into it).  A private range [lo, hi) must be whole parameters; ``last=False`` keeps
    the minibatch's copy count for the reductions of the other ranges (the overlapped data-parallel schedule)."""
    st = getattr(model, "_mdl_gws_buf", None)
    if st is None:
        return False
    ws, g, stride, copies = st
    hi = g.numel() if hi is None else hi
    if hi <= lo:
        return False
    if getattr(model, "_mdl_gws_mode", "atomic") == "private":
        grid = model._mdl_gws_grid
        if grid is None:   # no backward since the last reduction: nothing in the copies
            if not accumulate:
                g[lo:hi].zero_()
            return False
        if last:
            model._mdl_gws_grid = None
        fuse = norm_into is not None and lo == 0 and hi == g.numel()
        check(lib().mdl_grad_reduce_priv(g.data_ptr(), ws.data_ptr(), model._mdl_gws_dst.data_ptr(), lo, hi, stride,
                                         grid, int(bool(accumulate)), norm_into.data_ptr() if fuse else None,
                                         kernels._stream()), "grad_reduce_priv")
        return fuse
    if norm_into is not None and lo == 0 and hi == g.numel():
        check(lib().mdl_grad_reduce_norm(g.data_ptr(), ws.data_ptr(), hi, stride, copies, norm_into.data_ptr(),
                                         kernels._stream()), "grad_reduce_norm")
        return True
    check(lib().mdl_grad_reduce(g.data_ptr() + 4 * lo, ws.data_ptr() + 4 * lo, hi - lo, stride, copies,
                                kernels._stream()), "grad_reduce")
    return False


class UpdArgs(ctypes.Structure):   # csrc/ppo.hip mdl_update_fused
    _fields_ = [("g", VP), ("ws", VP), ("dst", VP), ("n", ctypes.c_int), ("stride", ctypes.c_longlong),
                ("copies", ctypes.c_int), ("accumulate", ctypes.c_int), ("a", AdamArgs), ("tab", VP),
                ("mat_off", VP), ("nmat", ctypes.c_int), ("rest", VP), ("n_rest", ctypes.c_int), ("bar", VP),
                ("ga", kernels.GatherArgs), ("ga_wg", ctypes.c_int)]


sig("mdl_update_fused", ctypes.POINTER(UpdArgs), VP)


class _UpdState:
    """Device tables of the fused update: the packed matrices' flat offsets, every other parameter element's flat
    index, and the grid barrier words."""

    def __init__(self, model, opt):
        mp = model_pack(model)
        lins = decoder_linears(model) + encoder_linears(model)
        base = opt.p.data_ptr()
        offs = [(l.weight.data_ptr() - base) // 4 for l in lins]
        n = opt.p.numel()
        is_mat = torch.zeros(n, dtype=torch.bool)
        for o in offs:
            assert 0 <= o and o + 4096 <= n
            is_mat[o:o + 4096] = True
        dev = opt.p.device
        self.mp = mp
        self.mat_off = torch.tensor(offs, dtype=torch.int32, device=dev)
        self.rest = torch.nonzero(~is_mat).flatten().to(torch.int32).to(dev)
        self.bar = torch.zeros(4, dtype=torch.int32, device=dev)
        self.nmat = len(offs)


def update_fused(model, opt, accumulate=False, gather=None):
    """Single-GPU end of a minibatch in TWO launches (csrc/ppo.hip mdl_update_fused: grad_reduce_priv +
    adam_pack): fold the private gradient workspace into the flat gradient with the Σ g² partials, then clip + Adam
    over every parameter and repack the 64 x 64 linears' bf16 fragments the training kernels read — replacing
    grad_reduce, adam_norm / adam_step and pack_weights (and the memset).  The caller bumps the model version; the
    ModelPack is marked current (its packs were written here).
    ``gather``: a ``kernels.gather_args`` struct — the NEXT minibatch's rows, gathered by extra workgroups of the
    adam_pack launch (rows <= 1024 floats wide), so the next minibatch starts without a gather launch of its own."""
    st = getattr(model, "_mdl_upd", None)
    if st is None or st.mp is not getattr(model, "_mdl_pack", None):
        st = _UpdState(model, opt)
        model._mdl_upd = st
    ws, g, stride, copies = model._mdl_gws_buf
    grid = model._mdl_gws_grid
    if grid is None:
        raise RuntimeError("update_fused: no backward wrote the private workspace this minibatch")
    model._mdl_gws_grid = None
    u = UpdArgs(g=g.data_ptr(), ws=ws.data_ptr(), dst=model._mdl_gws_dst.data_ptr(), n=g.numel(), stride=stride,
                copies=grid, accumulate=int(bool(accumulate)), a=opt.next_args(), tab=st.mp.table.data_ptr(),
                mat_off=st.mat_off.data_ptr(), nmat=st.nmat, rest=st.rest.data_ptr(), n_rest=st.rest.numel(),
                bar=st.bar.data_ptr())
    if gather is not None:
        u.ga = gather
    check(lib().mdl_update_fused(ctypes.byref(u), kernels._stream()), "update_fused")
    return st


def mark_packs_current(model):
    """After update_fused + bump_version: the ModelPack already holds the new weights' fragments."""
    mp = getattr(model, "_mdl_pack", None)
    if mp is not None:
        mp.version = getattr(model, "_mdl_version", 0)


def flat_range(params, flat):
    """[lo, hi) element range of ``flat`` holding the gradients of ``params`` (None if not one contiguous range)."""
    offs = sorted(((p.grad.data_ptr() - flat.data_ptr()) // 4, p.numel()) for p in params if p.grad is not None)
    if not offs:
        return None
    lo = end = offs[0][0]
    for o, n in offs:
        if not end <= o < end + 16:   # contiguous up to the per-parameter padding (ops/ppo_fused.PAD)
            return None
        end = o + n
    return lo, end


def _state(model, dev):
    st = getattr(model, "_mdl_train_state", None)
    if st is None:
        st = (EncoderFused(model), DecoderFused(model), torch.zeros((), device=dev, requires_grad=True))
        model._mdl_train_state = st
    return st


def evaluate_actions(model, obs, actions, ava=None):
    """Fused teacher-forced MAT forward with autograd support: (values, log-probs, entropy) like
    ``MultiAgentTransformer.forward``; gradients flow into the parameters' ``.grad``."""
    enc, dec, anchor = _state(model, obs.device)
    for p_ in model.parameters():
        if p_.grad is None:
            p_.grad = torch.zeros_like(p_)
    logp, v, ent = _MATFusedFn.apply(anchor, obs, actions, ava, enc, dec)
    return v, logp, ent


class _EncFusedFn(torch.autograd.Function):
    """(anchor, obs) -> (values, rep) through the fused encoder kernels; backward runs ``mat_enc_bwd`` with the
    rep gradient the eager decoder hands back.  The hybrid training path for models whose decoder is outside the
    fused gates (Available_Continuous, dec_actor, wide action heads): the encoder — the obs embedding and every
    encoder block — stays on the HIP kernels, only the decoder runs in autograd."""

    @staticmethod
    def forward(ctx, anchor, obs, enc):
        v, rep = enc.forward(obs, save=True)
        ctx.enc, ctx.saved = enc, enc.ctx   # this forward's activations (enc.ctx is shared, see _MATFusedFn)
        return v, rep

    @staticmethod
    def backward(ctx, dv, drep):
        enc = ctx.enc
        enc.ctx, ctx.saved = ctx.saved, None
        v, rep = enc.ctx[2], enc.ctx[1]
        enc.backward(drep if drep is not None else torch.zeros_like(rep),
                     dv if dv is not None else torch.zeros_like(v))
        enc.ctx = None
        return torch.zeros((), device=rep.device), None, None


def encode_train(model, obs):
    """Fused encoder forward with autograd: (values, rep) whose backward writes the encoder's parameter gradients
    straight into ``.grad`` (they are created zero-filled here when missing)."""
    enc, _, anchor = _state(model, obs.device)
    for p_ in model.encoder.parameters():
        if p_.grad is None:
            p_.grad = torch.zeros_like(p_)
    return _EncFusedFn.apply(anchor, obs, enc)


@torch.no_grad()
def encode(model, obs):
    """Inference-only fused encoder: (values, rep)."""
    enc, _, _ = _state(model, obs.device)
    return enc.forward(obs, save=False)
