"""Micro-benchmark of the fused training kernels on the bench minibatch shape (3200 sequences x 33 agents).

``python tests/bench_train_kernels.py [B] [L] [iters]`` (defaults 3200 33 10).
"""
import os
import sys
import time

import torch

sys.path.insert(0, "/root/repo/tests")
sys.path.insert(0, "/root/repo")
from test_gpu_train import make  # noqa: E402
from mat_dcml_amd.ops import mat_train  # noqa: E402


def main(B=3200, L=33, iters=10):
    dev = torch.device("cuda")
    m = make(L, dev, seed=0, scale=0.05)
    obs = torch.rand(B, L, 7, device=dev)
    ava = torch.ones(B, L, 2, device=dev)
    actions = (torch.rand(B, L, 1, device=dev) < 0.5).float()
    # the trainer's gradient layout: one flat fp32 buffer and its workspace (algos/mat_trainer.py): private
    # per-workgroup copies (round 6 default) or MAT_DCML_GRAD_MODE=atomic (32 shared copies, rounds 2-5)
    from mat_dcml_amd.ops import ppo_fused
    fp = ppo_fused.flatten_params(m)
    fg = torch.zeros_like(fp)
    for p, off in ppo_fused.param_offsets(m):
        p.grad = fg[off:off + p.numel()].view_as(p)
    copies = int(os.environ.get("MAT_DCML_GRAD_COPIES", "32"))
    mode = os.environ.get("MAT_DCML_GRAD_MODE", "private")
    if copies > 0:
        mat_train.attach_grad_workspace(m, fg, copies=copies, mode=mode)
    enc, dec = mat_train.EncoderFused(m), mat_train.DecoderFused(m)
    ev = {k: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for k in
          ("enc_fwd", "dec_fwd", "dec_bwd", "enc_bwd")}
    tot = {k: 0.0 for k in ev}
    for it in range(iters + 2):
        ev["enc_fwd"][0].record(); v, rep = enc.forward(obs); ev["enc_fwd"][1].record()
        ev["dec_fwd"][0].record(); lp, ent = dec.forward(rep, actions, ava); ev["dec_fwd"][1].record()
        m._mdl_gws_active = copies > 0
        ev["dec_bwd"][0].record(); drep = dec.backward(torch.ones_like(lp), torch.ones_like(ent)); ev["dec_bwd"][1].record()
        ev["enc_bwd"][0].record(); enc.backward(drep, torch.ones_like(v)); ev["enc_bwd"][1].record()
        m._mdl_gws_active = False
        if copies > 0:
            mat_train.reduce_grad_workspace(m, accumulate=False)
        torch.cuda.synchronize()
        if it >= 2:
            for k, (s, e) in ev.items():
                tot[k] += s.elapsed_time(e)
    print(f"B={B} L={L}: " + " | ".join(f"{k} {v / iters * 1e3:.0f} us" for k, v in tot.items())
          + f" | sum {sum(tot.values()) / iters * 1e3:.0f} us", flush=True)


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:]]
    main(*a)
