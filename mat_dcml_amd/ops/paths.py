"""Which compute path each hot op of a run takes — HIP kernel or eager PyTorch — and why a gate fell back.

The fused HIP paths have shape gates (``ops/mat_fused.unsupported_reasons``, ``ops/mat_train.*_unsupported_reasons``,
``MATTrainer.fused_reason``); a config outside them silently ran eager in round 1.  ``kernel_report`` makes the
choice visible: runners log it once at start-up and ``bench.py`` puts it in its JSON line.
"""
from __future__ import annotations

from . import kernels


def _hip(name, reasons):
    return f"hip:{name}" if not reasons else "torch (" + "; ".join(dict.fromkeys(reasons)) + ")"


def train_unsupported_reasons(model) -> list:
    """Why the fused training step (fused fwd/bwd + PPO loss + Adam) cannot run this model, device aside."""
    from . import mat_train
    r = mat_train.encoder_unsupported_reasons(model) + mat_train.decoder_unsupported_reasons(model)
    if getattr(model, "n_objective", 1) > 2:
        r.append(f"n_objective {model.n_objective} > 2")
    return list(dict.fromkeys(r))


def gate_reasons(model) -> dict:
    """Device-independent view of the fused gates: {op: [reasons]} ([] = the HIP kernel runs on a GPU)."""
    from . import mat_fused, mat_train
    return {"encoder": mat_train.encoder_unsupported_reasons(model), "decode": mat_fused.unsupported_reasons(model),
            "train": train_unsupported_reasons(model)}


def kernel_report(runner) -> dict:
    """{op: "hip:<kernel>" | "torch (<reason>)"} for the env step, rollout encoder, rollout decode, training
    forward/backward, GAE and the optimizer of a DCML / SMAC-style runner."""
    from . import mat_fused, mat_train
    pol = runner.policy
    dev = getattr(pol, "device", None)
    on_gpu = dev is not None and dev.type == "cuda"
    out = {}
    env = getattr(runner, "envs", None)
    if env is not None:
        kern = getattr(env, "_kern", None)
        if kern is not None:
            out["env"] = "hip:dcml_env_step"
        elif hasattr(env, "_kern"):
            out["env"] = "torch (" + ("cpu" if not on_gpu else f"backend={getattr(env, 'backend', '?')}") + ")"
        else:
            out["env"] = f"device env {type(env).__name__}"
    if not on_gpu:
        reason = ["cpu device"]
    elif getattr(pol, "kernels", "auto") == "torch" or kernels.mode() == "torch":
        reason = ["kernels=torch"]
    else:
        reason = []
    m = getattr(pol, "transformer", None)
    is_mat = hasattr(pol, "_is_mat") and pol._is_mat()
    if not is_mat:
        why = reason + [f"model {type(m).__name__} has no fused kernels"]
        out.update(encoder=_hip("", why), decode=_hip("", why), train=_hip("", why))
    else:
        out["encoder"] = _hip("mat_enc_fwd", reason or mat_train.encoder_unsupported_reasons(m))
        out["decode"] = _hip("mat_decode", reason or mat_fused.unsupported_reasons(m))
        if hasattr(m, "_mdl_decode_path") and out["decode"].startswith("hip:"):   # set by the last decode call
            out["decode"] += f"[{m._mdl_decode_path}]"
        tr = getattr(runner, "trainer", None)
        if tr is not None and getattr(tr, "fused", False):
            out["train"] = "hip:mat_enc_fwd/bwd+mat_dec_fwd/bwd+ppo_loss+adam"
        elif not reason and getattr(pol, "_enc_fused", lambda: False)() and mat_train.decoder_unsupported_reasons(m):
            # ops/mat_fused.evaluate_actions: fused encoder kernels under autograd, eager decoder
            out["train"] = "hybrid: hip:mat_enc_fwd/bwd + torch decoder (" + \
                "; ".join(mat_train.decoder_unsupported_reasons(m)) + ")"
        else:
            out["train"] = "torch (" + (getattr(tr, "fused_reason", None) or "; ".join(reason) or "eager") + ")"
    buf = getattr(runner, "buffer", None)
    if buf is not None:
        n_obj = getattr(buf, "n_objective", 1)
        why = list(reason)
        if getattr(buf, "use_advantage_norm", False):
            why.append("DMO normalised-advantage GAE")
        if n_obj > 1 and getattr(buf, "use_valuenorm", False) and not _gae_multi_objective():
            why.append("per-objective ValueNorm")
        out["gae"] = _hip("gae_reverse_scan", why)
    return out


def _gae_multi_objective():
    from . import rl_ops
    return getattr(rl_ops, "GAE_MULTI_OBJECTIVE", False)


def log_kernel_report(runner, stream=None):
    import sys
    rep = kernel_report(runner)
    if getattr(runner, "comm", None) is None or runner.comm.is_main:
        print("[kernels] " + ", ".join(f"{k}={v}" for k, v in rep.items()), file=stream or sys.stdout, flush=True)
    return rep
