"""Phase profile of the speculative decode (library built with -DMDL_SPEC_PROF, e.g.
MAT_DCML_LIBNAME=libmatdcml_ab_spprof.so MAT_DCML_DECW_FLAGS=-DMDL_SPEC_PROF python mat_dcml_amd/csrc/build.py):
s_memtime cycles per agent step of the main wave (block 1 / head / barrier wait) and the first speculative wave
(commit / block 0 / staging / barrier wait).   python scripts/spec_prof.py [L,nb,A,B ...]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from test_gpu_decode import inputs, make  # noqa: E402

from mat_dcml_amd.ops import mat_fused  # noqa: E402
from mat_dcml_amd.ops.kernels import lib  # noqa: E402

NAMES = {3: "main: setup (per launch / L)", 0: "main: barrier wait", 1: "main: slot read + block 1", 2: "main: head + sampling (rest)",
         8: "main: head W_h1 product", 9: "main: head GELU", 10: "main: head LN stats + split",
         11: "main: head logit MFMAs", 12: "main: sampling", 13: "main: action / log-prob stores",
         16 + 3: "spec: setup (per launch / L)", 16 + 4: "spec: barrier wait", 16 + 5: "spec: commit", 16 + 6: "spec: block 0", 16 + 7: "spec: staging"}


def main():
    shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or [(33, 2, 2, 256), (27, 2, 36, 32)]
    dev = torch.device("cuda:0")
    buf = (ctypes.c_ulonglong * 32)()
    fn = lib().mdl_spec_prof_read   # -DMDL_SPEC_PROF builds only
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for L, nb, A, B in shapes:
        m = make(L, dev, nb=nb, A=A, atype="Discrete" if A > 2 else "Semi_Discrete")
        obs, ava, rep, _ = inputs(m, B, L, dev, A=A)
        mat_fused.decode(m, rep, ava, False, 1, None)
        torch.cuda.synchronize()
        fn(ctypes.addressof(buf), 1)
        n = 10
        for _ in range(n):
            mat_fused.decode(m, rep, ava, False, 1, None)
        torch.cuda.synchronize()
        fn(ctypes.addressof(buf), 0)
        steps = n * B * L
        print(f"== {B}x{L} nb{nb} A{A} {m._mdl_decode_path}: cycles per agent step")
        for k, name in NAMES.items():
            print(f"   {name:28s} {buf[k] / steps:9.0f}")


if __name__ == "__main__":
    main()
