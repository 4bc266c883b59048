"""ctypes bindings for the in-tree HIP library ``mat_dcml_amd/_lib/libmatdcml.so`` (gfx950).

The library is plain HIP C++ (``mat_dcml_amd/csrc/*.hip``) compiled by ``hipcc --offload-arch=gfx950``
(``mat_dcml_amd/csrc/build.py``); each entry point takes raw device pointers and the current HIP stream,
so launches are captured by hipGraphs exactly like torch's own kernels.

Policy: on a GPU tensor the HIP path is the default and a missing library is an ERROR (no silent eager
fallback) unless ``MAT_DCML_KERNELS=torch`` is set explicitly.  CPU tensors always take the torch path.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "_lib", "libmatdcml.so")
_lib = None
_load_error = None


def mode():
    return os.environ.get("MAT_DCML_KERNELS", "auto").lower()


def lib():
    global _lib, _load_error
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            _load_error = f"{LIB_PATH} not built (run python -c 'import __graft_entry__ as g; g.build()')"
            raise RuntimeError(_load_error)
        _lib = ctypes.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


def available():
    if mode() == "torch":
        return False
    try:
        lib()
        return True
    except Exception:
        return False


def use_hip(t: torch.Tensor) -> bool:
    if not t.is_cuda or mode() == "torch":
        return False
    lib()  # raises loudly when the extension is missing on a GPU run
    return True


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def P(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


_SIGS = {}


def _declare(L):
    vp, i32, f32, i64, u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int64, ctypes.c_uint64
    for name, args in _SIGS.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int


def sig(name, *args):
    _SIGS[name] = list(args)


def check(rc, name):
    if rc != 0:
        raise RuntimeError(f"HIP kernel {name} failed with hipError {rc}")


# ----------------------------------------------------------------------------------------- RL ops
vp, i32, f32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int64
sig("mdl_gae_reverse_scan", vp, vp, vp, vp, vp, vp, i32, i32, f32, f32, vp)


def gae_reverse_scan(rewards, value_preds, masks, meanstd, gamma, lam, adv_out, ret_out):
    T = rewards.shape[0]
    n = rewards[0].numel()
    assert value_preds.shape[0] == T + 1 and masks.numel() == (T + 1) * n
    for t in (rewards, value_preds, masks, adv_out, ret_out):
        assert t.is_contiguous() and t.dtype == torch.float32
    check(lib().mdl_gae_reverse_scan(P(rewards), P(value_preds), P(masks), P(meanstd), P(adv_out), P(ret_out),
                                     T, n, gamma, lam, _stream()), "gae_reverse_scan")


u32 = ctypes.c_uint32
sig("mdl_philox_fill", vp, i32, u32, u32, u32, u32, u32, vp)


def philox_fill(n, c1, c2, c3, k0, k1, device):
    out = torch.empty(n, 4, dtype=torch.int64, device=device)
    check(lib().mdl_philox_fill(P(out), n, c1, c2, c3, k0, k1, _stream()), "philox_fill")
    return out
