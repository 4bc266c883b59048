"""One-shot peer-memory all-reduce across the ranks of one node (``csrc/xgmi_allreduce.hip``).

SURVEY.md §2.4: the data-parallel gradient is one 0.6 MB fp32 buffer per minibatch; a ring all-reduce over p GPUs
is 2(p−1) latency-bound hops over one xGMI link each, while the MI355X node is a full xGMI mesh.  Here every rank
exposes a shared region (two buffer halves + per-slice flags) through a HIP IPC handle; the handles are exchanged
once over the process group (any backend: the exchange is host-side ``all_gather_object``), every rank maps every
peer's region, and each all-reduce is ONE kernel launch on the current stream:
publish slice → flag every peer → wait for every peer's flag → sum the slice over ranks in rank order.

Results are bit-identical on every rank (fixed summation order).  Selected with ``MAT_DCML_ALLREDUCE=oneshot``
(forced) or ``=auto`` (``probe``: validated against ``dist.all_reduce`` and timed against it at start-up, kept only
if it agrees and is faster); RCCL stays the default (``Comm.maybe_enable_oneshot``).  Waits inside the kernel are
bounded: a peer that never arrives sets an error word instead of hanging the GPU, and ``check()`` raises on it.
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
        "mdl_ar_run": [ctypes.POINTER(_vp), _i32, _i32, _vp, _vp, _i64, _i32, _u32, _f32, _i64, _vp],
        "mdl_ar_error": [_vp, _i64, _i32, ctypes.POINTER(_u32)],
        "mdl_ar_error_async": [_vp, _i64, _i32, _vp, _vp],
    }.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    lib._mdl_ar_declared = True
    return lib


class OneShotAllReduce:
    """Peer-memory all-reduce of fp32 tensors of exactly ``n`` elements on ``comm``'s ranks.  Construction is
    collective and all-or-nothing: every rank runs the same collectives whatever fails locally, and if any rank
    cannot allocate / export / map a region, EVERY rank raises (so no rank is left on a different gradient path)."""

    def __init__(self, comm, n: int, n_wg: int = 0, wait_s: float = 120.0):
        if comm.device.type != "cuda":
            raise RuntimeError("one-shot all-reduce needs a GPU per rank")
        if not 1 <= comm.world_size <= MAX_WORLD:
            raise RuntimeError(f"one-shot all-reduce supports 1..{MAX_WORLD} ranks, got {comm.world_size}")
        self.comm, self.n = comm, int(n)
        # one workgroup per ~1.2k floats, at least 32 and at most 256 (one per CU): 0.6 MB -> 128 workgroups
        self.G = int(n_wg) or max(32, min(256, (self.n + 1183) // 1184))
        # bound of one in-kernel peer wait (shader clock <= 2.4 GHz): ranks legitimately drift apart by a whole
        # minibatch of compute, so this is a dead-peer guard, not a latency knob
        self.wait_cycles = int(wait_s * 2.4e9)
        self.lib = _declare(kernels.lib())
        self.own, self.opened, self.epoch, self.calls = None, [], 0, 0
        handle, err = None, ""
        with torch.cuda.device(comm.device):
            try:
                own = _vp()
                kernels.check(self.lib.mdl_ar_alloc(self.n, self.G, ctypes.byref(own)), "mdl_ar_alloc")
                self.own = own
                torch.cuda.synchronize(comm.device)
                hs = self.lib.mdl_ar_ipc_handle_size()
                buf = ctypes.create_string_buffer(hs)
                kernels.check(self.lib.mdl_ar_ipc_handle(own, buf), "mdl_ar_ipc_handle")
                handle = bytes(buf.raw)
            except Exception as e:   # keep going: the failure is reported collectively below
                err = repr(e)
            handles = comm.all_gather_object(handle)
            if any(h is None for h in handles):
                self._release()
                raise RuntimeError(f"one-shot all-reduce: region export failed on ranks "
                                   f"{[r for r, h in enumerate(handles) if h is None]} ({err or 'peer'})")
            self.regions = (_vp * comm.world_size)()
            ok = True
            try:
                for r, h in enumerate(handles):
                    if r == comm.rank:
                        self.regions[r] = self.own.value
                        continue
                    p = _vp()
                    kernels.check(self.lib.mdl_ar_open(ctypes.create_string_buffer(h, len(h)), ctypes.byref(p)),
                                  "mdl_ar_open")
                    self.regions[r] = p.value
                    self.opened.append(p)
            except Exception as e:
                ok, err = False, repr(e)
            oks = comm.all_gather_object(ok)
            if not all(oks):
                self._release()
                raise RuntimeError(f"one-shot all-reduce: mapping peer regions failed on ranks "
                                   f"{[r for r, o in enumerate(oks) if not o]} ({err or 'peer'})")
        comm.barrier()   # every region is zeroed and mapped before anyone signals

    def __call__(self, src: torch.Tensor, out: torch.Tensor | None = None, scale: float = 1.0) -> torch.Tensor:
        assert src.dtype == torch.float32 and src.is_contiguous() and src.numel() == self.n and src.is_cuda
        out = src if out is None else out
        assert out.dtype == torch.float32 and out.is_contiguous() and out.numel() == self.n
        self.epoch += 1
        self.calls += 1
        rc = self.lib.mdl_ar_run(self.regions, self.comm.world_size, self.comm.rank, _vp(src.data_ptr()),
                                 _vp(out.data_ptr()), self.n, self.G, self.epoch, float(scale), self.wait_cycles,
                                 _vp(torch.cuda.current_stream().cuda_stream))
        kernels.check(rc, "mdl_ar_run")
        return out

    def error_word(self) -> int:
        v = _u32(0)
        kernels.check(self.lib.mdl_ar_error(self.own, self.n, self.G, ctypes.byref(v)), "mdl_ar_error")
        return int(v.value)

    def poll(self):
        """Asynchronous error check, once per training iteration: raise if the error word copied by the PREVIOUS
        poll (on the current stream, into pinned memory) is set, then queue the next copy.  A timed-out wait also
        wrote NaN over its output slice, so the optimizer has already skipped that step; this turns it into a
        loud failure one iteration later without a device synchronisation.  The timed-out rank also set bit 31 of
        every peer's word (csrc/xgmi_allreduce.hip), so the peers whose own waits succeeded raise here as well."""
        if getattr(self, "_err_host", None) is None:
            self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self._err_ev = None
        if self._err_ev is not None and self._err_ev.query() and int(self._err_host[0]):
            raise RuntimeError(f"rank {self.comm.rank}: one-shot all-reduce peer wait timed out "
                               f"(mask {int(self._err_host[0]) & 0xffffffff:#x})")
        if self._err_ev is None or self._err_ev.query():
            st = torch.cuda.current_stream()
            kernels.check(self.lib.mdl_ar_error_async(self.own, self.n, self.G, _vp(self._err_host.data_ptr()),
                                                      _vp(st.cuda_stream)), "mdl_ar_error_async")
            self._err_ev = torch.cuda.Event()
            self._err_ev.record(st)

    def check(self):
        """Synchronous: raise if any wait inside the kernel timed out since the region was created."""
        e = self.error_word()
        if e:
            raise RuntimeError(f"rank {self.comm.rank}: one-shot all-reduce peer wait timed out (mask {e:#x})")

    def _release(self):
        for p in self.opened:
            self.lib.mdl_ar_close(p)
        self.opened = []
        if self.own is not None:
            self.lib.mdl_ar_free(self.own)
            self.own = None

    def close(self):
        torch.cuda.synchronize(self.comm.device)
        self.comm.barrier()   # nobody still reads a region we are about to unmap / free
        self._release()


def probe(comm, n: int, iters: int = 20, margin: float = 0.95):
    """Collective: build the one-shot all-reduce for n floats, check it against ``dist.all_reduce`` (the process
    group's backend: RCCL on a GPU node) on random data and time both back to back (median per call, max over
    ranks).  Returns (chosen, OneShotAllReduce or None, info):
    one-shot is chosen only if it agrees with RCCL and is faster by ``margin``; every rank takes the same decision."""
    import torch.distributed as dist
    info = {"n": int(n)}
    try:
        ar = OneShotAllReduce(comm, n)
    except RuntimeError as e:   # raised on every rank together
        info["error"] = str(e)
        return "rccl", None, info
    dev = comm.device
    g = torch.Generator(device="cpu").manual_seed(12345 + comm.rank)
    x = torch.randn(n, generator=g).to(dev)
    y1 = torch.empty_like(x)
    ar(x, out=y1)
    y2 = x.clone()
    dist.all_reduce(y2, group=comm.group)
    torch.cuda.synchronize(dev)
    err = float((y1 - y2).abs().max() / y2.abs().max().clamp_min(1e-30))
    ok = err <= 1e-5 and ar.error_word() == 0

    def timed(fn):
        comm.barrier()
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(iters):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            ts.append((a, b))
        torch.cuda.synchronize(dev)
        v = sorted(a.elapsed_time(b) * 1e3 for a, b in ts)
        return v[len(v) // 2]

    t_os = timed(lambda: ar(y1, scale=1.0 / comm.world_size))
    t_rc = timed(lambda: dist.all_reduce(y2, group=comm.group))
    ok = ok and ar.error_word() == 0
    rows = comm.all_gather_object((ok, err, t_os, t_rc))
    info.update(agree=all(r[0] for r in rows), max_rel_err=max(r[1] for r in rows), backend=comm.backend,
                oneshot_us=round(max(r[2] for r in rows), 2), backend_us=round(max(r[3] for r in rows), 2))
    if info["agree"] and info["oneshot_us"] < margin * info["backend_us"]:
        return "oneshot", ar, info
    ar.close()
    return "rccl", None, info
