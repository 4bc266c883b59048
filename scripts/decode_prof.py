"""Per-phase cycle breakdown of the persistent decode kernel (workgroup 0, thread 0), rollout shape.
Run with MAT_DCML_LIBNAME=libmatdcml_prof.so (built with -DMDL_DECODE_PROF)."""
import ctypes
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from test_gpu_train import make, make_discrete  # noqa: E402

from mat_dcml_amd.ops import kernels, mat_fused  # noqa: E402

NAMES = ["pass setup", "A qkv", "B self-attn", "C proj1", "D kv2/q2", "E cross-attn", "F proj2", "G mlp1",
         "H mlp2", "I head1", "J head/sample", "K token update"]
dev = torch.device("cuda")
CASES = [("DCML 256 x 33", 33, 256, None), ("DCML 256 x 101", 101, 256, None), ("SMAC 32 x 27, 36 actions", 27, 32, 36)]
for name, L, B, A in CASES:
    if A is None:
        m = make(L, dev, seed=0, scale=0.05)
        obs = torch.rand(B, L, 7, device=dev)
        ava = torch.ones(B, L, 2, device=dev)
    else:   # the SMAC-shaped head: Discrete(36) with availability (the decode does not see the 1288-wide obs)
        m = make_discrete(L, A, 16, dev, seed=0, scale=0.05)
        obs = torch.rand(B, L, 16, device=dev)
        ava = (torch.rand(B, L, A, device=dev) < 0.7).float()
        ava[..., 0] = 1.0
    with torch.no_grad():
        for _ in range(3):
            mat_fused.get_actions(m, obs, ava, False, 1, None)
    torch.cuda.synchronize()
    out = (ctypes.c_ulonglong * 24)()
    lib = kernels.lib()
    lib.mdl_decode_prof_read.argtypes = [ctypes.c_void_p]
    assert lib.mdl_decode_prof_read(ctypes.addressof(out)) == 0
    tot = sum(out[:12])
    print(f"{name}: L={L}: {tot} cycles total ({tot / L:.0f} per agent)")
    for k, n in enumerate(NAMES):
        print(f"  {n:16s} {out[k]:10d} {100 * out[k] / max(tot, 1):5.1f}%  {out[k] / L:8.0f}/agent")
    print("  phase G sub-marks (12: since the previous sub-mark / barrier, 13: afrag_ln, 14: store_xf + MFMA, "
          "15: GELU + XA stores):", [out[k] for k in (12, 13, 14, 15)])
