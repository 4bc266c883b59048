"""One-shot peer-memory all-reduce across the ranks of one node (``csrc/xgmi_allreduce.hip``).

SURVEY.md §2.4: the data-parallel gradient is one 0.6 MB fp32 buffer per minibatch; a ring all-reduce over p GPUs
is 2(p−1) latency-bound hops over one xGMI link each, while the MI355X node is a full xGMI mesh.  Here every rank
exposes a shared region (two buffer halves + per-slice flags) through a HIP IPC handle; the handles are exchanged
once over the process group (any backend: the exchange is host-side ``all_gather_object``), every rank maps every
peer's region, and each all-reduce is ONE kernel launch on the current stream:
publish slice → flag every peer → wait for every peer's flag → sum the slice over ranks in rank order.

Results are bit-identical on every rank (fixed summation order).  Selected with ``MAT_DCML_ALLREDUCE=oneshot``
(``Comm.enable_oneshot``); RCCL stays the default.  Waits inside the kernel are bounded: a peer that never arrives
sets an error word instead of hanging the GPU, and ``check()`` raises on it.
"""
from __future__ import annotations

import ctypes

import torch

from ..ops import kernels

_vp, _i32, _i64, _u32, _f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint32, ctypes.c_float
MAX_WORLD = 16


def _declare(lib):
    if getattr(lib, "_mdl_ar_declared", False):
        return lib
    for name, args in {
        "mdl_ar_alloc": [_i64, _i32, ctypes.POINTER(_vp)],
        "mdl_ar_free": [_vp],
        "mdl_ar_ipc_handle_size": [],
        "mdl_ar_ipc_handle": [_vp, ctypes.c_char_p],
        "mdl_ar_open": [ctypes.c_char_p, ctypes.POINTER(_vp)],
        "mdl_ar_close": [_vp],
        "mdl_ar_run": [ctypes.POINTER(_vp), _i32, _i32, _vp, _vp, _i64, _i32, _u32, _f32, _i32, _vp],
        "mdl_ar_error": [_vp, _i64, _i32, ctypes.POINTER(_u32)],
    }.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    lib._mdl_ar_declared = True
    return lib


class OneShotAllReduce:
    """Peer-memory all-reduce of fp32 tensors of exactly ``n`` elements on ``comm``'s ranks (collective
    construction: every rank must build it, in the same order)."""

    def __init__(self, comm, n: int, n_wg: int = 0, spin_max: int = 1_000_000):
        if comm.device.type != "cuda":
            raise RuntimeError("one-shot all-reduce needs a GPU per rank")
        if not 1 <= comm.world_size <= MAX_WORLD:
            raise RuntimeError(f"one-shot all-reduce supports 1..{MAX_WORLD} ranks, got {comm.world_size}")
        self.comm, self.n = comm, int(n)
        # one workgroup per ~1.2k floats, at least 32 and at most 256 (one per CU): 0.6 MB -> 128 workgroups
        self.G = int(n_wg) or max(32, min(256, (self.n + 1183) // 1184))
        self.spin_max = int(spin_max)
        self.lib = _declare(kernels.lib())
        with torch.cuda.device(comm.device):
            own = _vp()
            kernels.check(self.lib.mdl_ar_alloc(self.n, self.G, ctypes.byref(own)), "mdl_ar_alloc")
            torch.cuda.synchronize(comm.device)
            hs = self.lib.mdl_ar_ipc_handle_size()
            buf = ctypes.create_string_buffer(hs)
            kernels.check(self.lib.mdl_ar_ipc_handle(own, buf), "mdl_ar_ipc_handle")
            handles = comm.all_gather_object(bytes(buf.raw))
            self.own = own
            self.regions = (_vp * comm.world_size)()
            self.opened = []
            for r, h in enumerate(handles):
                if r == comm.rank:
                    self.regions[r] = own.value
                    continue
                p = _vp()
                kernels.check(self.lib.mdl_ar_open(ctypes.create_string_buffer(h, hs), ctypes.byref(p)), "mdl_ar_open")
                self.regions[r] = p.value
                self.opened.append(p)
        comm.barrier()   # every region is zeroed and mapped before anyone signals
        self.epoch = 0
        self.calls = 0

    def __call__(self, src: torch.Tensor, out: torch.Tensor | None = None, scale: float = 1.0) -> torch.Tensor:
        assert src.dtype == torch.float32 and src.is_contiguous() and src.numel() == self.n and src.is_cuda
        out = src if out is None else out
        assert out.dtype == torch.float32 and out.is_contiguous() and out.numel() == self.n
        self.epoch += 1
        self.calls += 1
        rc = self.lib.mdl_ar_run(self.regions, self.comm.world_size, self.comm.rank, _vp(src.data_ptr()),
                                 _vp(out.data_ptr()), self.n, self.G, self.epoch, float(scale), self.spin_max,
                                 _vp(torch.cuda.current_stream().cuda_stream))
        kernels.check(rc, "mdl_ar_run")
        return out

    def error_word(self) -> int:
        v = _u32(0)
        kernels.check(self.lib.mdl_ar_error(self.own, self.n, self.G, ctypes.byref(v)), "mdl_ar_error")
        return int(v.value)

    def check(self):
        """Synchronous: raise if any wait inside the kernel timed out since the region was created."""
        e = self.error_word()
        if e:
            raise RuntimeError(f"rank {self.comm.rank}: one-shot all-reduce peer wait timed out (mask {e:#x})")

    def close(self):
        torch.cuda.synchronize(self.comm.device)
        self.comm.barrier()   # nobody still reads a region we are about to unmap / free
        for p in self.opened:
            self.lib.mdl_ar_close(p)
        self.opened = []
        if self.own is not None:
            self.lib.mdl_ar_free(self.own)
            self.own = None
