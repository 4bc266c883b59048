"""One-wave decode debugging: per-row log-prob error vs teacher forcing across L, and (with the -DMDL_WAVE_DEBUG
library, MAT_DCML_LIBNAME=libmatdcml_wdbg.so) the kernel's intermediates of env 0 / row R vs the torch decoder."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from test_gpu_decode import inputs, make  # noqa: E402

from mat_dcml_amd.models import act  # noqa: E402
from mat_dcml_amd.ops import kernels, mat_fused  # noqa: E402

dev = torch.device("cuda")
NAMES = ["x_in", "O_self", "x1", "O_cross", "x2", "x3"]


def intermediates(m, rep, obs, a, row):
    dec = m.decoder
    got = {}
    hooks = []

    def out_hook(name):
        return lambda mod, inp, out: got.__setitem__(name, out[0, row].float().clone())

    def in_hook(name):
        return lambda mod, inp: got.__setitem__(name, inp[0][0, row].float().clone())

    hooks.append(dec.ln.register_forward_hook(out_hook("b0.x_in")))
    for b, blk in enumerate(dec.blocks):
        hooks.append(blk.attn1.proj.register_forward_pre_hook(in_hook(f"b{b}.O_self")))
        hooks.append(blk.ln1.register_forward_hook(out_hook(f"b{b}.x1")))
        hooks.append(blk.attn2.proj.register_forward_pre_hook(in_hook(f"b{b}.O_cross")))
        hooks.append(blk.ln2.register_forward_hook(out_hook(f"b{b}.x2")))
        hooks.append(blk.ln3.register_forward_hook(out_hook(f"b{b}.x3")))
        if b + 1 < len(dec.blocks):
            hooks.append(blk.ln3.register_forward_hook(out_hook(f"b{b + 1}.x_in")))
    hooks.append(dec.head[1].register_forward_hook(out_hook("head.h")))
    hooks.append(dec.head.register_forward_hook(out_hook("head.logits")))
    with torch.no_grad():
        dec(act.shifted_from_actions(m, a).to(rep.dtype), rep, obs)
    for h in hooks:
        h.remove()
    return got


def per_row():
    for atype, L, nb in [("Discrete", 40, 2), ("Semi_Discrete", 33, 2), ("Discrete", 70, 1)]:
        m = make(L, dev, atype=atype, seed=11, nb=nb)
        obs, ava, rep, rand = inputs(m, 64, L, dev)
        ava = torch.ones_like(ava)
        for wave in (True, False):
            mat_fused.WAVE_DECODE = wave
            a, lp = mat_fused.decode(m, rep, ava, False, 1, rand)
            with torch.no_grad():
                lp_tf, _ = act.parallel_act(m, rep, obs, a, ava)
            err = (lp_tf - lp).abs().mean(0).view(-1)
            bad = [(i, round(e, 3)) for i, e in enumerate(err.tolist()) if e > 5e-3]
            print(atype, "L", L, "nb", nb, m._mdl_decode_path, "bad rows:", bad[:8], flush=True)


def stages(L=33, nb=2, rows=(0,)):
    lib = kernels.lib()
    fn = lib.mdl_wave_debug_read
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    m = make(L, dev, atype="Semi_Discrete", seed=11, nb=nb)
    obs, ava, rep, rand = inputs(m, 8, L, dev)
    ava = torch.ones_like(ava)
    mat_fused.WAVE_DECODE = True
    buf = (ctypes.c_float * (16 * 64))()
    for row in rows:
        assert fn(None, row) == 0
        a, lp = mat_fused.decode(m, rep, ava, False, 1, rand)
        torch.cuda.synchronize()
        assert fn(ctypes.addressof(buf), -1) == 0
        k = torch.tensor(list(buf)).view(16, 64)
        ref = intermediates(m, rep, obs, a, row)
        print(f"--- row {row} ({m._mdl_decode_path})")
        for b in range(nb):
            for j, nm in enumerate(NAMES):
                r = ref.get(f"b{b}.{nm}")
                kk = k[6 * b + j]
                print(f"  b{b}.{nm:8s} max|ref| {r.abs().max().item():8.4f}  max|err| {(kk - r.cpu()).abs().max().item():9.5f}"
                      f"  first {kk[:4].tolist()} ref {r[:4].cpu().tolist()}")
        r = ref["head.h"]
        print(f"  head.h     max|err| {(k[12] - r.cpu()).abs().max().item():9.5f}")
        r = ref["head.logits"]
        A = r.shape[0]
        print(f"  logits     kernel {k[13][:A].tolist()} ref {r.cpu().tolist()}")


if __name__ == "__main__":
    if os.environ.get("MAT_DCML_LIBNAME", "").endswith("wdbg.so"):
        stages()
    else:
        per_row()
