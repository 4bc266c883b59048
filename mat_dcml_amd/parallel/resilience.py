"""Failure detection, fault injection and elastic restart.

The reference has no rank failures to handle (it is single-process) and no health checks: a hung env blocks
``step_wait`` forever (``env_wrappers.py:373``).  Here:

* ``Heartbeat`` — each rank publishes a timestamp into the ``torch.distributed`` TCPStore every ``period`` s from a
  daemon thread; rank 0's watchdog declares a rank dead when its heartbeat is older than ``timeout`` and aborts the
  job (``os._exit``), which the launcher turns into a restart.  Collective timeouts come from
  ``init_process_group(timeout=…)`` (RCCL watchdog).
* ``FaultInjector`` — test hooks from ``--fault_inject``: ``nan@<it>`` poisons the gradients of iteration ``it``
  (exercises the non-finite guard that skips the optimizer step), ``kill@<rank>:<it>`` hard-exits that rank at
  iteration ``it`` (exercises restart-from-checkpoint), ``disable@<frac>`` forces the env's disabled-worker
  fraction.  Several specs can be joined with commas.
* ``launch_with_restarts`` — runs the training command as a child process (never ``exec``) and relaunches it with
  ``--resume`` up to ``max_restarts`` times after a failure; the trainer then restores weights, Adam moments,
  ValueNorm statistics, the episode counter and each rank's env counters from the latest checkpoint.
"""
from __future__ import annotations

import os
import subprocess
import sys
import threading
import time

import torch
import torch.distributed as dist

KILL_EXIT_CODE = 17


class FaultInjector:
    def __init__(self, spec: str | None, rank: int = 0):
        self.rank = rank
        self.nan_at, self.kill_at, self.disable_frac = set(), None, None
        for part in (spec or "").split(","):
            part = part.strip()
            if not part:
                continue
            kind, _, arg = part.partition("@")
            if kind == "nan":
                self.nan_at.add(int(arg))
            elif kind == "kill":
                r, _, it = arg.partition(":")
                if int(r) == rank:
                    self.kill_at = int(it)
            elif kind == "disable":
                self.disable_frac = float(arg)
            else:
                raise ValueError(f"unknown fault spec {part!r}")

    def poison_grads(self, iteration: int) -> bool:
        return iteration in self.nan_at

    def maybe_kill(self, iteration: int, before=None):
        """Injected hard kill at ``iteration``; ``before()`` (e.g. the runner's pending-log flush) runs first."""
        if self.kill_at is not None and iteration == self.kill_at:
            if before is not None:
                before()
            print(f"[fault_inject] rank {self.rank}: killed at iteration {iteration}", file=sys.stderr, flush=True)
            sys.stdout.flush()   # os._exit skips the interpreter's buffer flush
            os._exit(KILL_EXIT_CODE)


class Heartbeat:
    def __init__(self, comm, period_s: float, timeout_s: float | None = None):
        self.comm = comm
        self.period = float(period_s)
        self.timeout = float(timeout_s or max(10 * period_s, 30.0))
        self.store = None
        self._stop = threading.Event()
        self.dead = []
        if self.period <= 0 or comm.world_size == 1 or not dist.is_initialized():
            return
        try:
            self.store = dist.distributed_c10d._get_default_store()
        except Exception:   # noqa: BLE001 — no store: heartbeats disabled
            self.store = None
            return
        self._beat()
        threading.Thread(target=self._loop, daemon=True).start()

    def _beat(self):
        self.store.set(f"mdl_hb/{self.comm.rank}", repr(time.time()))

    def _loop(self):
        while not self._stop.wait(self.period):
            try:
                self._beat()
                if self.comm.rank == 0:
                    self.check()
            except Exception:   # noqa: BLE001 — store gone: the job is shutting down
                return

    def check(self):
        now = time.time()
        dead = []
        for r in range(self.comm.world_size):
            try:
                t = float(self.store.get(f"mdl_hb/{r}").decode())
            except Exception:   # noqa: BLE001
                continue
            if now - t > self.timeout:
                dead.append(r)
        self.dead = dead
        if dead:
            print(f"[heartbeat] ranks {dead} silent for > {self.timeout:.0f}s: aborting for restart",
                  file=sys.stderr, flush=True)
            os._exit(KILL_EXIT_CODE + 1)
        return dead

    def stop(self):
        self._stop.set()


def grads_finite(flat_buf: torch.Tensor) -> torch.Tensor:
    """Device bool (no host sync) — used by the torch path; the fused Adam kernel skips non-finite steps itself."""
    return torch.isfinite(flat_buf).all()


def launch_with_restarts(cmd: list[str], max_restarts: int, env=None) -> int:
    """Run ``cmd``; on a non-zero exit relaunch it with ``--resume`` (at most ``max_restarts`` times)."""
    attempt = 0
    while True:
        run = list(cmd) + (["--resume"] if attempt > 0 and "--resume" not in cmd else [])
        print(f"[launcher] attempt {attempt}: {' '.join(run)}", flush=True)
        rc = subprocess.call(run, env=env)
        if rc == 0 or attempt >= max_restarts:
            return rc
        attempt += 1
        print(f"[launcher] exit code {rc}: restarting from the latest checkpoint ({attempt}/{max_restarts})",
              flush=True)


def main(argv=None):
    """``python -m mat_dcml_amd.parallel.resilience --max_restarts 2 -- <training command …>``"""
    argv = list(sys.argv[1:] if argv is None else argv)
    n = 0
    if "--max_restarts" in argv:
        i = argv.index("--max_restarts")
        n = int(argv[i + 1])
        del argv[i:i + 2]
    if argv and argv[0] == "--":
        argv = argv[1:]
    return launch_with_restarts(argv, n)


if __name__ == "__main__":
    sys.exit(main())
