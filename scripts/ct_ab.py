"""A/B timing of the CT training kernels (one library per process, MAT_DCML_LIBNAME): enc/dec forward + backward at
the bench minibatch shape (3200 x 33), hipEvent-timed, median of N repetitions."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from test_gpu_train import make  # noqa: E402

from mat_dcml_amd.ops import mat_train  # noqa: E402


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main(B=3200, L=33, reps=20):
    dev = torch.device("cuda")
    m = make(L, dev, seed=0, scale=0.05)
    obs = torch.rand(B, L, 7, device=dev)
    ava = torch.ones(B, L, 2, device=dev)
    actions = (torch.rand(B, L, 1, device=dev) < 0.5).float()
    from mat_dcml_amd.parallel.comm import FlatGrads
    fg = FlatGrads(list(m.parameters()))   # the trainer's layout: .grad views of one flat buffer + 8-copy workspace
    mat_train.attach_grad_workspace(m, fg.buf, copies=int(os.environ.get("MAT_DCML_GRAD_COPIES", "32")))
    m._mdl_gws_active = True
    enc, dec = mat_train.EncoderFused(m), mat_train.DecoderFused(m)
    st = {}
    v, rep = enc.forward(obs)
    lp, ent = dec.forward(rep, actions, ava)
    drep = dec.backward(torch.ones_like(lp), torch.ones_like(ent))
    enc.backward(drep, torch.ones_like(v))
    torch.cuda.synchronize()
    st["enc_fwd"] = timed(lambda: enc.forward(obs), reps)
    st["dec_fwd"] = timed(lambda: dec.forward(rep, actions, ava), reps)
    st["dec_bwd"] = timed(lambda: dec.backward(torch.ones_like(lp), torch.ones_like(ent)), reps)
    st["enc_bwd"] = timed(lambda: enc.backward(drep, torch.ones_like(v)), reps)
    st["grad_reduce"] = timed(lambda: mat_train.reduce_grad_workspace(m), reps)
    st["total"] = sum(st.values())
    print(os.environ.get("MAT_DCML_LIBNAME", "libmatdcml.so"), f"B={B} L={L}",
          " ".join(f"{k} {v:.1f}us" for k, v in st.items()))


if __name__ == "__main__":
    for L in os.environ.get("CT_AB_L", "33").split(","):
        L = int(L)
        main(B=3200 * 33 // L if L != 33 else 3200, L=L)
