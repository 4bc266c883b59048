"""Fused PPO loss/gradients and flat clip+Adam (``csrc/ppo.hip``) + flat parameter storage.

* ``flatten_params(module)``: every parameter becomes a view of ONE contiguous fp32 buffer (same order as
  ``FlatGrads`` in ``parallel/comm.py``), so the optimizer is a single elementwise kernel over 151k floats
  and the gradient all-reduce / norm / clip see one buffer.
* ``FlatAdam``: ``torch.optim.Adam`` semantics (bias-corrected moments, eps outside the sqrt, L2 weight decay)
  fused with ``clip_grad_norm_`` (scale = min(1, max_norm / (‖g‖ + 1e-6))) — 1 memset + 2 kernels instead of the
  ~25 launches of foreach-Adam + clip.  ``param_groups`` / ``state_dict`` keep the optimizer-facing surface
  (``lr_decay``, checkpoints).
* ``ppo_loss``: the MAT-PPO objective's value and analytic gradients w.r.t. (values, log-probs, entropies) in
  3 kernels, including the ValueNorm update (reference ``mat_trainer.py:54-156``); its outputs feed the fused
  decoder / encoder backward kernels directly (``ops/mat_train.py``).
"""
from __future__ import annotations

import ctypes
import warnings

import torch

from . import kernels
from .kernels import P, _stream, check, lib, sig

vp = ctypes.c_void_p


class PPOArgs(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("n_obj", ctypes.c_int)] + \
               [(k, vp) for k in ("v", "logp", "ent", "old_logp", "adv", "vpred", "ret", "active", "dv", "dlogp",
                                  "dent", "stats", "out", "vn")] + \
               [(k, ctypes.c_float) for k in ("clip", "coef_v", "coef_e", "huber_delta", "beta", "eps", "omb")] + \
               [(k, ctypes.c_int) for k in ("use_huber", "use_clip_v", "use_vam", "use_pam", "use_vn", "update_vn",
                                            "n_lp")] + \
               [("sidx", vp), ("L", ctypes.c_int), ("adv_sums", vp), ("adv_eps", ctypes.c_float)]


class AdamArgs(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int)] + [(k, vp) for k in ("p", "g", "m", "v", "sumsq")] + \
               [(k, ctypes.c_float) for k in ("lr", "beta1", "beta2", "eps", "wd", "t", "max_norm")] + \
               [("clip", ctypes.c_int), ("npart", ctypes.c_int)]


sig("mdl_ppo_loss", ctypes.POINTER(PPOArgs), vp)
sig("mdl_ppo_reduce", ctypes.POINTER(PPOArgs), vp)
sig("mdl_ppo_finish", ctypes.POINTER(PPOArgs), vp)
sig("mdl_ppo_finish_fused", ctypes.POINTER(PPOArgs), vp, vp)
sig("mdl_adam", ctypes.POINTER(AdamArgs), ctypes.c_int, vp)


PAD = 16   # every parameter starts on a 64-byte boundary of the flat buffer (aligned float4 loads in the kernels)


def padded(n: int) -> int:
    return (n + PAD - 1) // PAD * PAD


def flatten_params(module: torch.nn.Module) -> torch.Tensor:
    """Move every trainable parameter into ONE flat fp32 buffer (views), each padded to 16 floats.  The padding
    stays zero: its gradient is never written, so Adam leaves it at zero."""
    params = [p for p in module.parameters() if p.requires_grad]
    n = sum(padded(p.numel()) for p in params)
    dev = params[0].device
    flat = torch.zeros(n, dtype=torch.float32, device=dev)
    off = 0
    for p in params:
        k = p.numel()
        flat[off:off + k].copy_(p.data.reshape(-1).float())
        p.data = flat[off:off + k].view_as(p)
        off += padded(k)
    module._mdl_flat_params = flat
    return flat


def flat_params_of(module):
    flat = getattr(module, "_mdl_flat_params", None)
    if flat is None:
        return None
    params = [p for p in module.parameters() if p.requires_grad]
    off = 0
    for p in params:   # views still in place (load_state_dict copies into them)
        if p.data_ptr() != flat[off:].data_ptr():
            return None
        off += padded(p.numel())
    return flat


def param_offsets(module):
    """[(param, offset)] of the flat layout (same for the flat parameters and the flat gradients)."""
    out, off = [], 0
    for p in module.parameters():
        if p.requires_grad:
            out.append((p, off))
            off += padded(p.numel())
    return out


def _adam_scratch_floats():
    try:
        return int(lib().mdl_adam_scratch_floats())
    except Exception:   # CPU-only state handling without the library: same layout (4 + ADAM_NB)
        return 4 + 1024


class FlatAdam:
    """Adam + clip over the flat buffers.  The step counter used for the bias corrections is the number of APPLIED
    steps (attempted ``t`` minus the device-side count of skipped non-finite steps), like ``torch.optim.Adam``.
    ``state_dict`` is torch.optim.Adam's per-parameter format, so a fused-path checkpoint resumes on the eager
    path (and vice versa)."""

    def __init__(self, flat_params: torch.Tensor, flat_grads: torch.Tensor, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0, max_grad_norm=None, layout=None):
        self.p, self.g = flat_params, flat_grads
        self.m = torch.zeros_like(flat_params)
        self.v = torch.zeros_like(flat_params)
        # [1] grad norm, [2] skipped steps, [3] Σ norms (logging), [4:] per-workgroup Σ g² partials (csrc/ppo.hip)
        self.scratch = torch.zeros(_adam_scratch_floats(), dtype=torch.float32, device=flat_params.device)
        self.param_groups = [{"lr": lr, "betas": betas, "eps": eps, "weight_decay": weight_decay}]
        self.max_grad_norm = max_grad_norm
        self.layout = layout   # [(param, flat offset)] (ops/ppo_fused.param_offsets)
        self.t = 0

    @property
    def grad_norm(self):
        return self.scratch[1]

    @property
    def grad_norm_sum(self):
        """Σ of the step norms since ``clear_grad_norm_sum`` (accumulated in-kernel: no add launch per step)."""
        return self.scratch[3]

    def clear_grad_norm_sum(self):
        self.scratch[3:4].zero_()

    @property
    def skipped_steps(self):
        return self.scratch[2]

    def zero_grad(self, set_to_none=False):
        self.g.zero_()

    def next_args(self):
        """AdamArgs of the next step (advances the attempted-step counter)."""
        g = self.param_groups[0]
        self.t += 1
        b1, b2 = g["betas"]
        return AdamArgs(n=self.p.numel(), p=P(self.p), g=P(self.g), m=P(self.m), v=P(self.v), sumsq=P(self.scratch),
                        lr=g["lr"], beta1=b1, beta2=b2, eps=g["eps"], wd=g["weight_decay"], t=float(self.t),
                        max_norm=float(self.max_grad_norm or 0.0), clip=int(self.max_grad_norm is not None), npart=0)

    def step(self, norm_ready=False):
        """``norm_ready``: the Σ g² partials of this step's gradient are already in the scratch
        (``mat_train.reduce_grad_workspace(..., norm_into=self.scratch)``): no norm launch."""
        a = self.next_args()
        check(lib().mdl_adam(ctypes.byref(a), int(bool(norm_ready)), _stream()), "adam")

    def applied_steps(self) -> int:
        return self.t - int(round(float(self.scratch[2])))

    def state_dict(self):
        grp = {k: v for k, v in self.param_groups[0].items()}
        grp.update(amsgrad=False, maximize=False, foreach=None, capturable=False, differentiable=False, fused=None)
        if self.layout is None:
            raise RuntimeError("FlatAdam.state_dict needs the parameter layout")
        step = float(self.applied_steps())
        state = {}
        for i, (p, off) in enumerate(self.layout):
            n = p.numel()
            state[i] = {"step": torch.tensor(step), "exp_avg": self.m[off:off + n].view_as(p).detach().clone(),
                        "exp_avg_sq": self.v[off:off + n].view_as(p).detach().clone()}
        grp["params"] = list(range(len(self.layout)))
        return {"state": state, "param_groups": [grp]}

    def load_state_dict(self, sd):
        if "m" in sd:   # round-1 flat format: the parameters concatenated WITHOUT the per-parameter padding
            m_old, v_old = sd["m"].reshape(-1), sd["v"].reshape(-1)
            self.m.zero_()
            self.v.zero_()
            if m_old.numel() == self.m.numel():
                self.m.copy_(m_old)
                self.v.copy_(v_old)
                self.t = int(sd["t"])
            elif self.layout is not None and m_old.numel() == sum(p.numel() for p, _ in self.layout):
                o = 0   # remap the unpadded moments through the padded layout
                for p, off in self.layout:
                    n = p.numel()
                    self.m[off:off + n].copy_(m_old[o:o + n].to(self.m.device))
                    self.v[off:off + n].copy_(v_old[o:o + n].to(self.v.device))
                    o += n
                self.t = int(sd["t"])
            else:   # moments unusable: restart them AND the bias-correction step count (a large t with zero
                warnings.warn("FlatAdam: legacy optimizer state does not match the parameter layout; "   # moments
                              "Adam moments and step count reset")                                     # = 3x steps)
                self.t = 0
            self.scratch[2] = 0.0
            self.param_groups[0].update({k: v for k, v in sd["param_groups"][0].items() if k != "params"})
            return
        st = sd.get("state", {})
        if st:
            if self.layout is None or len(self.layout) != len(st):
                raise RuntimeError("optimizer state does not match the model's parameters")
            self.m.zero_()
            self.v.zero_()
            for i, (p, off) in enumerate(self.layout):
                n = p.numel()
                self.m[off:off + n].copy_(st[i]["exp_avg"].reshape(-1).to(self.m.device))
                self.v[off:off + n].copy_(st[i]["exp_avg_sq"].reshape(-1).to(self.v.device))
            self.t = int(float(st[min(st)]["step"]))
            self.scratch[2] = 0.0
        self.param_groups[0]["lr"] = sd["param_groups"][0]["lr"]


class PPOLossFused:
    """Holds the per-trainer device scratch; ``run`` launches the fused loss for one minibatch."""

    def __init__(self, trainer, device):
        self.tr = trainer
        self.stats = torch.zeros(8, dtype=torch.float32, device=device)
        self.out = torch.zeros(4, dtype=torch.float32, device=device)
        self._vn = None
        self._g = None
        self._ctr = torch.zeros(1, dtype=torch.int32, device=device)   # ppo_finish_fused's arrival counter

    def _vn_buffer(self, n_obj, device):
        """ValueNorm moments as views of one flat buffer the kernels update in place (bound once)."""
        vnm = self.tr.value_normalizer
        if vnm is None:
            if self._vn is None:
                self._vn = torch.zeros(2 * n_obj + 1, dtype=torch.float32, device=device)
            return self._vn
        flat = getattr(vnm, "_mdl_flat", None)
        if flat is None or vnm.running_mean.data_ptr() != flat.data_ptr():
            flat = torch.cat([vnm.running_mean.reshape(-1), vnm.running_mean_sq.reshape(-1),
                              vnm.debiasing_term.reshape(-1)]).float().contiguous()
            shp_m, shp_d = vnm.running_mean.shape, vnm.debiasing_term.shape
            vnm.running_mean = flat[:n_obj].view(shp_m)
            vnm.running_mean_sq = flat[n_obj:2 * n_obj].view(shp_m)
            vnm.debiasing_term = flat[2 * n_obj].view(shp_d)
            vnm._mdl_flat = flat
        return flat

    def run(self, values, logp, ent, mb, comm=None, pre_stats=None):
        """values (N, n_obj), logp / ent (N, 1) fp32 contiguous → (dv, dlogp, dent).  Losses accumulate into
        ``self.out`` = [policy, value, entropy, ratio] (caller zeroes it per log window)."""
        tr = self.tr
        n_obj = values.shape[-1]
        N = values.numel() // n_obj           # tokens
        n_lp = logp.numel() // N              # log-prob entries per token (continuous: action dims)
        dev = values.device
        if self._g is None or self._g[0].shape != values.shape or self._g[1].shape != logp.shape:
            self._g = (torch.empty_like(values), torch.empty_like(logp), torch.empty_like(ent))
        dv, dlp, dent = self._g
        vnm = tr.value_normalizer
        vn = self._vn_buffer(n_obj, dev)
        ts = [t.reshape(-1).contiguous() if t.is_contiguous() else t.contiguous() for t in
              (mb["old_logp"], mb["adv"], mb["value_preds"], mb["returns"], mb["active"])]
        stats = self.stats if pre_stats is None else pre_stats
        # round 6: mb may carry the rollout buffer's rows + the epoch permutation ("idx") and the advantage sums
        # ("adv_sums"): the kernels read through the index and standardise the advantages themselves (no gather)
        idx, adv_sums = mb.get("idx"), mb.get("adv_sums")
        L = values.shape[1] if values.dim() == 3 else 1
        a = PPOArgs(n=N, n_obj=n_obj, v=P(values), logp=P(logp), ent=P(ent), old_logp=P(ts[0]), adv=P(ts[1]),
                    vpred=P(ts[2]), ret=P(ts[3]), active=P(ts[4]), dv=P(dv), dlogp=P(dlp), dent=P(dent),
                    stats=P(stats), out=P(self.out), vn=P(vn), clip=tr.clip_param, coef_v=tr.value_loss_coef,
                    coef_e=tr.entropy_coef, huber_delta=tr.huber_delta, beta=vnm.beta if vnm is not None else 1.0,
                    eps=vnm.epsilon if vnm is not None else 1e-5,
                    omb=(1.0 - vnm.beta) if vnm is not None else 0.0, use_huber=int(tr._use_huber_loss),
                    use_clip_v=int(tr._use_clipped_value_loss), use_vam=int(tr._use_value_active_masks),
                    use_pam=int(tr._use_policy_active_masks), use_vn=int(vnm is not None),
                    update_vn=int(vnm is not None), n_lp=n_lp, sidx=P(idx) if idx is not None else None, L=L,
                    adv_sums=P(adv_sums) if adv_sums is not None else None, adv_eps=1e-5)
        if idx is not None:
            assert idx.dtype == torch.int64 and idx.is_contiguous() and idx.numel() * L == N
        if adv_sums is not None:
            assert adv_sums.dtype == torch.float64
        if pre_stats is not None:   # statistics of this minibatch precomputed (and all-reduced) for the epoch
            assert pre_stats.dtype == torch.float32 and pre_stats.numel() == 2 * n_obj + 2 and pre_stats.is_contiguous()
            # ValueNorm update + loss gradients in one launch (round 6)
            check(lib().mdl_ppo_finish_fused(ctypes.byref(a), P(self._ctr), _stream()), "ppo_finish_fused")
        elif comm is not None and comm.world_size > 1 and vnm is not None:
            check(lib().mdl_ppo_reduce(ctypes.byref(a), _stream()), "ppo_reduce")
            comm.all_reduce_sum_(self.stats[: 2 * n_obj + 1])
            check(lib().mdl_ppo_finish(ctypes.byref(a), _stream()), "ppo_finish")
        else:
            check(lib().mdl_ppo_loss(ctypes.byref(a), _stream()), "ppo_loss")
        return dv, dlp, dent


def available():
    return kernels.available()
