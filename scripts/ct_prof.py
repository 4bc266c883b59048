"""Phase profile of the CT training kernels (build with -DMDL_CT_PROF, scripts/ct_prof.sh): s_memtime cycles per
phase summed over every workgroup, one kernel at a time, at the bench minibatch shape (3200 x 33)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from test_gpu_train import make  # noqa: E402

from mat_dcml_amd.ops import kernels, mat_train  # noqa: E402

NAMES = {0: "tile start (zero LDS)", 1: "head bwd (tiles)", 19: "head bwd wgrads", 2: "mlp bwd tiles",
         3: "mlp bwd wgrads", 4: "cross bwd proj+LN", 6: "cross recompute qkv + wgrad proj",
         7: "cross attn bwd q", 8: "cross attn bwd kv", 9: "cross stage rep/x1 + dX + drep", 10: "cross wgrad qkv",
         11: "self bwd proj+LN", 13: "self recompute qkv + wgrad proj", 14: "self attn bwd q (+ stage x)",
         15: "self attn bwd kv", 16: "self dX", 17: "self wgrad qkv", 30: "embedding bwd",
         20: "self qkv fwd", 21: "self attn fwd", 22: "self proj+LN fwd", 23: "mlp fwd (wave 0)", 24: "cross qkv fwd",
         25: "cross attn fwd", 26: "cross proj+LN fwd", 27: "head fwd (rest)", 28: "embedding fwd",
         31: "head fwd: weight loads", 32: "head fwd: W_h1 + GELU + LN + saves", 33: "head fwd: logits",
         34: "head fwd: softmax stats + stores"}


def read(fn):
    out = (ctypes.c_ulonglong * 64)()
    assert fn(ctypes.addressof(out), 0) == 0
    assert fn(ctypes.addressof(out), 1) == 0
    return list(out)


def main(B=3200, L=33, reps=3):
    dev = torch.device("cuda")
    lib = kernels.lib()
    for n in ("mdl_ctprof_enc", "mdl_ctprof_dec", "mdl_ctprof_enc_bwd", "mdl_ctprof_dec_bwd"):
        getattr(lib, n).argtypes = [ctypes.c_void_p, ctypes.c_int]
    # the backward kernels live in their own translation units (mat_*_ct_bwd.hip) with their own counters
    penc, pdec, penc_b, pdec_b = lib.mdl_ctprof_enc, lib.mdl_ctprof_dec, lib.mdl_ctprof_enc_bwd, lib.mdl_ctprof_dec_bwd
    m = make(L, dev, seed=0, scale=0.05)
    obs = torch.rand(B, L, 7, device=dev)
    ava = torch.ones(B, L, 2, device=dev)
    actions = (torch.rand(B, L, 1, device=dev) < 0.5).float()
    for p in m.parameters():
        p.grad = torch.zeros_like(p)
    enc, dec = mat_train.EncoderFused(m), mat_train.DecoderFused(m)
    res = {}
    for r in range(reps + 1):
        read(penc), read(pdec), read(penc_b), read(pdec_b)
        v, rep = enc.forward(obs); torch.cuda.synchronize(); a = read(penc)
        lp, ent = dec.forward(rep, actions, ava); torch.cuda.synchronize(); b = read(pdec)
        drep = dec.backward(torch.ones_like(lp), torch.ones_like(ent)); torch.cuda.synchronize(); c = read(pdec_b)
        enc.backward(drep, torch.ones_like(v)); torch.cuda.synchronize(); d = read(penc_b)
        if r:
            for name, arr in (("enc_fwd", a), ("dec_fwd", b), ("dec_bwd", c), ("enc_bwd", d)):
                acc = res.setdefault(name, [0] * 64)
                for i in range(64):
                    acc[i] += arr[i]
    for name, acc in res.items():
        tot = sum(acc[:63])
        print(f"{name}: {tot / reps / 1e6:.2f} M cycles summed over workgroups")
        for i in sorted(range(63), key=lambda i: -acc[i]):
            if acc[i]:
                print(f"   {NAMES.get(i, str(i)):28s} {100 * acc[i] / tot:5.1f}%")


if __name__ == "__main__":
    main()
