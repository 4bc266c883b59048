"""Per-phase cycle breakdown of the persistent decode kernel (workgroup 0, thread 0), rollout shape.
Run with MAT_DCML_LIBNAME=libmatdcml_prof.so (built with -DMDL_DECODE_PROF)."""
import ctypes
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from test_gpu_train import make  # noqa: E402

from mat_dcml_amd.ops import kernels, mat_fused  # noqa: E402

NAMES = ["pass setup", "A qkv", "B self-attn", "C proj1", "D kv2/q2", "E cross-attn", "F proj2", "G mlp1",
         "H mlp2", "I head1", "J head/sample", "K token update"]
dev = torch.device("cuda")
for L in (33, 101):
    m = make(L, dev, seed=0, scale=0.05)
    obs = torch.rand(256, L, 7, device=dev)
    ava = torch.ones(256, L, 2, device=dev)
    with torch.no_grad():
        for _ in range(3):
            mat_fused.get_actions(m, obs, ava, False, 1, None)
    torch.cuda.synchronize()
    out = (ctypes.c_ulonglong * 24)()
    lib = kernels.lib()
    lib.mdl_decode_prof_read.argtypes = [ctypes.c_void_p]
    assert lib.mdl_decode_prof_read(ctypes.addressof(out)) == 0
    tot = sum(out[:12])
    print(f"L={L}: {tot} cycles total ({tot / L:.0f} per agent)")
    for k, n in enumerate(NAMES):
        print(f"  {n:16s} {out[k]:10d} {100 * out[k] / max(tot, 1):5.1f}%  {out[k] / L:8.0f}/agent")
    print("  phase G sub-marks (12: since the previous sub-mark / barrier, 13: afrag_ln, 14: store_xf + MFMA, "
          "15: GELU + XA stores):", [out[k] for k in (12, 13, 14, 15)])
