"""Decode-path bisection for the rollout-vs-learner log-prob gap: one rollout step's observations, the same explicit
random draws through every decode kernel (speculative / one-wave / 4-wave) and the fp32 torch autoregressive decode;
each kernel's log-probs against the learner's teacher-forced ones on that kernel's own actions.

    python scripts/logprob_diag2.py [--ckpt ...]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ckpt", default="profiles/r5_train32/transformer_500_beta3.pt")
    ap.add_argument("--n_workers", type=int, default=32)
    a = ap.parse_args()
    from test_gpu_logprob_consistency import _dcml_runner
    from mat_dcml_amd.models import act
    from mat_dcml_amd.ops import mat_fused, mat_train
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    r = _dcml_runner(dev, a.n_workers, 256, 2)
    if a.ckpt:
        r.policy.restore(a.ckpt)
    m = r.policy.transformer
    r.warmup()
    r.rollout()
    b = r.buffer
    obs, ava = b.obs[1].contiguous(), b.available_actions[1].contiguous()
    B, L = obs.shape[:2]
    g = torch.Generator(device=dev).manual_seed(5)
    rand = {"u": torch.rand(B, L, device=dev, generator=g), "n": torch.randn(B, L, m.action_dim, device=dev, generator=g)}
    enc, dec, _ = mat_train._state(m, dev)
    with torch.no_grad():
        v, rep = mat_fused._encode(m, obs)
        a_t, lp_t = act.autoregressive_act(m, rep, obs, ava, False, 1, rand)

    def learner(acts):
        with torch.no_grad():
            _, rp = enc.forward(obs, save=True)
            lp, _ = dec.forward(rp, acts, ava, save=True)
            tf, _ = act.parallel_act(m, rep, obs, acts, ava)
        return lp.reshape(B, L, -1), tf.reshape(B, L, -1).float()

    saved = mat_fused.WAVE_DECODE, mat_fused.SPEC_DECODE
    try:
        for name, wave, spec in (("spec", True, True), ("wave", True, False), ("4wave", False, False)):
            mat_fused.WAVE_DECODE, mat_fused.SPEC_DECODE = wave, spec
            with torch.no_grad():
                ak, lpk = mat_fused.decode(m, rep, ava, False, 1, rand)
            torch.cuda.synchronize()
            path = m._mdl_decode_path
            lr, tf = learner(ak)
            d = (lpk.reshape(B, L, -1) - lr).abs()
            dt = (lpk.reshape(B, L, -1) - tf).abs()
            agree = (ak[:, :L - 1] == a_t[:, :L - 1]).float().mean().item()
            print(f"{name} [{path}]: vs learner mean {d.mean().item():.3e} max {d.max().item():.3e}; vs fp32 TF mean "
                  f"{dt.mean().item():.3e} max {dt.max().item():.3e}; actions agree with torch decode {agree:.4f}; "
                  f"per-row mean (first 4) {[round(x, 4) for x in d.mean((0, 2))[:4].tolist()]}")
    finally:
        mat_fused.WAVE_DECODE, mat_fused.SPEC_DECODE = saved
    with torch.no_grad():
        lr, tf = learner(a_t)
    print(f"torch decode: vs learner mean {(lp_t.reshape(B, L, -1) - lr).abs().mean().item():.3e}")


if __name__ == "__main__":
    main()
