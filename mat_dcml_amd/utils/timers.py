"""Phase timers (hipEvent based on GPU) and roctx ranges.

The reference only prints wall-clock FPS (``dcml_runner.py:96-104``) and eval inference time
(``:337-345,445``).  Here every phase (decode / env / insert / update / allreduce) can be bracketed:

* ``PhaseTimers`` records a pair of ``torch.cuda.Event`` per phase occurrence and resolves them lazily
  (one sync at ``summary()``), so enabling it does not serialise the pipeline;
* ``roctx`` ranges (``librocprofiler-sdk-roctx.so``) mark the same phases in ``rocprofv3 --marker-trace``.
"""
from __future__ import annotations

import contextlib
import ctypes
import time

import torch

_roctx = None


def _load_roctx():
    global _roctx
    if _roctx is None:
        for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so"):
            try:
                _roctx = ctypes.CDLL(name)
                _roctx.roctxRangePushA.argtypes = [ctypes.c_char_p]
                break
            except OSError:
                continue
        else:
            _roctx = False
    return _roctx


@contextlib.contextmanager
def roctx_range(name: str):
    lib = _load_roctx()
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


class PhaseTimers:
    """``every``: {phase: n} records only every n-th occurrence of a frequent phase and scales its total by
    occurrences / recorded (bench.py: each recorded hipEvent pair costs a few microseconds of stream bubble, so the
    per-rollout-step and per-minibatch phases are sampled to keep the timed loop within 1 % of its untimed speed)."""

    def __init__(self, device, enabled=False, every=None):
        self.enabled = enabled
        self.cuda = torch.device(device).type == "cuda"
        self.events = {}
        self.host = {}
        self.every = dict(every or {})
        self.count = {}

    @contextlib.contextmanager
    def __call__(self, name):
        if not self.enabled:
            yield
            return
        n = self.count.get(name, 0)
        self.count[name] = n + 1
        if n % self.every.get(name, 1):
            yield
            return
        with roctx_range(name):
            if self.cuda:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                yield
                e.record()
                self.events.setdefault(name, []).append((s, e))
            else:
                t = time.perf_counter()
                yield
                self.host.setdefault(name, []).append(time.perf_counter() - t)

    def totals_ms(self):
        out = {k: sum(v) * 1e3 * self.count.get(k, len(v)) / len(v) for k, v in self.host.items()}
        if self.events:
            torch.cuda.synchronize()
            for k, v in self.events.items():
                out[k] = out.get(k, 0.0) + sum(s.elapsed_time(e) for s, e in v) * self.count.get(k, len(v)) / len(v)
        return out

    def summary(self, reset=True):
        tot = self.totals_ms()
        s = " | ".join(f"{k} {v:.1f} ms" for k, v in tot.items())
        if reset:
            self.events.clear()
            self.host.clear()
            self.count.clear()
        return "[phases] " + s
