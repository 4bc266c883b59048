"""Data-parallel communicator: one process per GPU, RCCL over xGMI (``torch.distributed`` backend ``nccl``).

The reference has no distributed training at all (no torch.distributed / NCCL / MPI; device
hard-coded to ``cuda:0``).  This module is the new DP layer:

* ``init_from_env`` — reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (torchrun contract),
  binds ``cuda:LOCAL_RANK`` and creates the process group (``nccl`` = RCCL on ROCm; ``gloo`` for CPU tests).
* ``FlatGrads`` — every parameter's ``.grad`` is a view into ONE contiguous fp32 buffer (151k floats ≈ 606 KB
  for the DCML MAT), so a data-parallel gradient average is ONE all-reduce with no pack/unpack copies.
  At this message size a ring all-reduce over xGMI is latency-bound (2(p−1) hops); one bucket per minibatch is
  the right granularity — splitting it into per-layer buckets to overlap with backward only adds latency.
* ``all_reduce_sum_`` for the small statistics vectors (advantage moments, ValueNorm moments, metrics),
  packed by the callers into one message each.
* ``grad_mean_`` averages the flat gradient: RCCL by default, or the one-shot peer-memory kernel over the xGMI
  mesh (``parallel/oneshot.py``, ``csrc/xgmi_allreduce.hip``) with ``MAT_DCML_ALLREDUCE=oneshot``.
"""
from __future__ import annotations

import contextlib
import datetime
import os
import socket
import time

import torch
import torch.distributed as dist


class Comm:
    def __init__(self, rank=0, world_size=1, local_rank=0, device=torch.device("cpu"), group=None):
        self.rank, self.world_size, self.local_rank = rank, world_size, local_rank
        self.device = device
        self.group = group
        self._flat = None
        self.backend = "none"
        self.oneshot = None          # OneShotAllReduce of the flat gradient (opt-in)
        self.oneshot_probe = None    # start-up check / timing of the one-shot path (mode "auto")
        self._timing = None          # {name: [event pairs | seconds]} while enable_timing(True)
        # MAT_DCML_ALLREDUCE=ordered: gradients by all-gather + rank-order sum (see _ordered_sum_)
        self.ordered = os.environ.get("MAT_DCML_ALLREDUCE", "").lower() == "ordered"

    # -------------------------------------------------------------------------------- timing (bench.py)
    def enable_timing(self, on: bool = True):
        """Time every critical-path collective (flat-gradient average, statistics all-reduces) on the current
        stream: hipEvents before / after, so the time includes waiting for the slowest rank."""
        self._timing = {} if on else None

    @contextlib.contextmanager
    def _timed(self, name):
        if self._timing is None or self.world_size == 1:
            yield
            return
        if self.device.type == "cuda":
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            yield
            b.record()
            self._timing.setdefault(name, []).append((a, b))
        else:
            t0 = time.perf_counter()
            yield
            self._timing.setdefault(name, []).append(time.perf_counter() - t0)

    def timing_ms(self, reset: bool = True) -> dict:
        """{name: total ms, name + "_calls": count} since the last reset (synchronise the device first)."""
        out = {}
        for k, v in (self._timing or {}).items():
            out[k] = round(sum(x[0].elapsed_time(x[1]) if isinstance(x, tuple) else x * 1e3 for x in v), 4)
            out[k + "_calls"] = len(v)
        if reset and self._timing is not None:
            self._timing = {}
        return out

    @property
    def is_main(self):
        return self.rank == 0

    # -------------------------------------------------------------------------------- collectives
    def all_reduce_sum_(self, t: torch.Tensor):
        if self.world_size > 1:
            with self._timed("stats_allreduce"):
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def grad_sum_(self, t: torch.Tensor):
        """SUM all-reduce of a gradient slice, timed as gradient traffic (the overlapped schedule's remaining range)."""
        if self.world_size > 1:
            with self._timed("grad_allreduce"):
                if self.ordered:
                    self._ordered_sum_(t)
                else:
                    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    # ordered gradient reduction (MAT_DCML_ALLREDUCE=ordered): all-gather, then a rank-order sum on every rank.  A ring
    # all-reduce sums each element in an order set by the message's chunking, so the same gradient all-reduced as one
    # buffer or as two slices can differ in the last bit at >= 3 ranks; the ordered sum does not depend on how the
    # buffer is split (the overlapped schedule is then bitwise the blocking one) and is identical on every rank
    ordered = False

    def _gather(self, t, async_op=False):
        out = torch.empty(self.world_size * t.numel(), dtype=t.dtype, device=t.device)
        w = dist.all_gather_into_tensor(out, t.contiguous().view(-1), group=self.group, async_op=async_op)
        return out.view(self.world_size, -1), w

    @staticmethod
    def _fold(t, out):
        acc = out[0].clone()
        for r in range(1, out.shape[0]):
            acc += out[r]
        t.copy_(acc.view_as(t))
        return t

    def _ordered_sum_(self, t):
        out, _ = self._gather(t)
        return self._fold(t, out)

    def all_reduce_max_(self, t: torch.Tensor):
        if self.world_size > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t

    def all_reduce_mean_(self, t: torch.Tensor):
        if self.world_size > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            t.div_(self.world_size)
        return t

    def barrier(self):
        if self.world_size > 1:
            if self.device.type == "cuda":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)

    def broadcast_module_(self, module: torch.nn.Module, src=0):
        if self.world_size > 1:
            with torch.no_grad():
                for t in list(module.parameters()) + list(module.buffers()):
                    dist.broadcast(t.data, src=src, group=self.group)

    def all_gather_object(self, obj):
        if self.world_size == 1:
            return [obj]
        out = [None] * self.world_size
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def seed_sampling_rng(self, seed: int):
        """Call after the (identical, broadcast) weight init: every rank gets its own torch RNG stream, so the
        rollout's exploration draws (decode uniforms / normals) are independent across ranks instead of repeating
        rank 0's noise in every replica."""
        torch.manual_seed(int(seed) + 1_000_003 * self.rank)

    # -------------------------------------------------------------------------------- gradients
    def attach_flat_grads(self, params):
        self._flat = FlatGrads(params)
        return self._flat

    def all_reduce_grads_(self, params):
        if self.world_size == 1:
            return
        if self._flat is None or not self._flat.owns(params):
            self.attach_flat_grads(params)
        self._flat.ensure_views()
        self.grad_mean_(self._flat.buf)

    def grad_mean_(self, buf: torch.Tensor):
        """Average the flat gradient buffer over ranks in place: one kernel launch with the one-shot peer-memory
        all-reduce when enabled for this buffer size (the 1/world scale is applied in-kernel), else RCCL."""
        if self.world_size == 1:
            return buf
        with self._timed("grad_allreduce"):
            if self.oneshot is not None and buf.numel() == self.oneshot.n and buf.is_cuda:
                return self.oneshot(buf, scale=1.0 / self.world_size)
            if self.ordered:
                self._ordered_sum_(buf)
            else:
                dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)
            return buf.mul_(1.0 / self.world_size)

    def maybe_enable_oneshot(self, n: int, mode: str | None = None):
        """Collective: pick the flat-gradient all-reduce for n-float gradients.  ``MAT_DCML_ALLREDUCE`` (or ``mode``):
        ``rccl`` (default), ``oneshot`` (forced; every rank raises together if it cannot be built) or ``auto``
        (``oneshot.probe``: kept only when it matches RCCL and is faster).  Returns the selected path."""
        mode = (mode or os.environ.get("MAT_DCML_ALLREDUCE", "rccl")).lower()
        if self.world_size == 1:
            return "none"
        if mode == "ordered":
            self.ordered = True
            return "ordered"
        if mode not in ("oneshot", "auto") or self.device.type != "cuda":
            return self.backend
        if self.oneshot is not None and self.oneshot.n == n:
            return "oneshot"
        from . import oneshot
        if mode == "oneshot":
            self.oneshot = oneshot.OneShotAllReduce(self, n)
            return "oneshot"
        chosen, ar, self.oneshot_probe = oneshot.probe(self, n)
        self.oneshot = ar
        return "oneshot" if chosen == "oneshot" else self.backend

    def poll_errors(self):
        """Once per training iteration, without a device sync: raise if a one-shot all-reduce peer wait timed out
        (its NaN output already made the optimizer skip that step; see ``OneShotAllReduce.poll``)."""
        if self.oneshot is not None:
            self.oneshot.poll()

    def all_reduce_sum_async(self, t: torch.Tensor, grad=False):
        """Start a SUM all-reduce of ``t``; returns a work handle (``wait()`` makes the current stream wait) or None.
        With the nccl (RCCL) backend the collective runs on the process group's own HIP stream, ordered after the
        work already queued on the current stream, so kernels launched afterwards overlap it.  ``grad``: a gradient
        slice (the ordered reduction applies, folded into ``t`` at ``wait()``)."""
        if self.world_size == 1:
            return None
        if grad and self.ordered:
            out, w = self._gather(t, async_op=True)
            fold = self._fold

            class _Work:
                def wait(self_):
                    w.wait()
                    fold(t, out)
            return _Work()
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def describe(self) -> dict:
        """Gathered rank → device map of the job (collective: every rank must call it).  ``distinct_devices`` counts
        physical devices (host, device index); CPU ranks count as one device each."""
        if self.device.type == "cuda":
            me = (socket.gethostname(), f"cuda:{self.device.index}")
        else:
            me = (socket.gethostname(), f"cpu:rank{self.rank}")
        allv = self.all_gather_object(me)
        return {"backend": self.backend, "world_size": self.world_size, "devices": [d for _, d in allv],
                "hosts": sorted({h for h, _ in allv}), "distinct_devices": len(set(allv)),
                "shared_devices": len(set(allv)) < self.world_size}

    def destroy(self):
        if self.oneshot is not None:
            ar, self.oneshot = self.oneshot, None
            try:
                ar.check()   # a timed-out peer wait anywhere in the run fails the run loudly
            finally:
                ar.close()
        if self.world_size > 1 and dist.is_initialized():
            dist.destroy_process_group()


class FlatGrads:
    """All ``.grad`` tensors as views of one flat buffer (zero_grad must use ``set_to_none=False``)."""

    PAD = 16   # same per-parameter padding as the flat parameter buffer (ops/ppo_fused.flatten_params)

    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        pad = lambda k: (k + self.PAD - 1) // self.PAD * self.PAD  # noqa: E731
        n = sum(pad(p.numel()) for p in self.params)
        dev = self.params[0].device
        self.buf = torch.zeros(n, dtype=torch.float32, device=dev)
        self.views = []
        off = 0
        for p in self.params:
            v = self.buf[off:off + p.numel()].view_as(p)
            if p.grad is not None:
                v.copy_(p.grad)
            p.grad = v
            self.views.append(v)
            off += pad(p.numel())
        self._ids = {id(p) for p in self.params}

    def owns(self, params):
        return all(id(p) in self._ids for p in params if p.requires_grad)

    def ensure_views(self):
        for p, v in zip(self.params, self.views):
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                if p.grad is not None:
                    v.copy_(p.grad)
                else:
                    v.zero_()
                p.grad = v


def init_from_env(prefer_gpu=True, timeout_s=600, share_devices=None) -> Comm:
    """One process per device.  Under RCCL (``nccl``) every rank must own its own GPU: a LOCAL_RANK beyond the
    visible device count is an error.  Sharing one GPU between ranks (rehearsals on a 1-GPU box) is an explicit
    opt-in (``share_devices=True`` or ``MAT_DCML_SHARE_DEVICES=1``) and is allowed with the gloo backend only."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = prefer_gpu and torch.cuda.is_available()
    backend = os.environ.get("MAT_DCML_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    if share_devices is None:
        share_devices = os.environ.get("MAT_DCML_SHARE_DEVICES", "0") == "1"
    device = torch.device("cpu")
    if use_gpu:
        ndev = torch.cuda.device_count()
        if local >= ndev:
            if not share_devices or backend == "nccl":
                raise RuntimeError(
                    f"rank {rank}: LOCAL_RANK {local} but only {ndev} visible GPU(s); backend {backend!r} needs one GPU "
                    f"per rank (device sharing is opt-in via MAT_DCML_SHARE_DEVICES=1 and only with gloo)")
            device = torch.device(f"cuda:{local % ndev}")
        else:
            device = torch.device(f"cuda:{local}")
        torch.cuda.set_device(device)
    group = None
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if use_gpu and backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    c = Comm(rank, world, local, device, group)
    c.backend = backend if world > 1 else "none"
    return c
