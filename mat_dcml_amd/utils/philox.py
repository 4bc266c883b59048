"""Counter-based Philox4x32-10 random streams, bit-identical to the HIP device version.

The reference draws from Python ``random`` / ``np.random`` inside forked env processes and is
irreproducible by construction (``DCML_BID_FIRST_MA_ENV_SingleProcess.py:158-199``,
``DCML_Worker_TIMESLOT_MultiProcess.py:53-59``).  Every random draw in this framework is instead a pure
function of ``(seed, counter)``: the counter is ``(episode_step, global_env_id, sub, purpose)``, so a
1-GPU run and an 8-GPU run over the same global env set produce identical rollouts.

This module is the torch (CPU / fallback) implementation.  ``csrc/common.h`` holds the device version;
``tests/test_philox.py`` pins them against each other and against published Philox test vectors.
All uint32 arithmetic is carried in int64 tensors and masked.
"""
from __future__ import annotations

import torch

M0 = 0xD2511F53
M1 = 0xCD9E8D57
W0 = 0x9E3779B9
W1 = 0xBB67AE85
MASK32 = 0xFFFFFFFF

# Purpose ids (counter word 3).  Shared with csrc/dcml_env.hip — keep in sync.
P_MASTER = 1        # R, C, master Pr, disable count
P_ARRIVE = 2        # arrive time, done draw, disable-subset keys base
P_WORKER_PR = 3     # per-worker loss probability
P_NOISE = 4         # per-worker workload noise (5 calls x 4 words = 20 slots)
P_DISABLE = 5       # per-worker random key for the disabled subset
P_DOWNLOAD = 6      # per-worker download retries
P_UPLOAD = 7        # per-worker upload retries, sub = slot iteration
P_DONE = 8          # per-env done draw
P_SHANNON = 9       # Shannon link draws (distance, worker power; sub 0xFFFF = master power)
P_POLICY = 16       # policy sampling streams (decode kernel)
P_SMAC = 32         # SMAC-shaped env battle resets (csrc/smac_env.hip)


def _mulhilo(a: int, b: torch.Tensor):
    prod = b * a  # int64 wraps modulo 2^64: low 64 bits are exact
    lo = prod & MASK32
    hi = (prod >> 32) & MASK32
    return hi, lo


def philox4x32(c0, c1, c2, c3, k0: int, k1: int, rounds: int = 10):
    """Philox4x32-``rounds`` on int64 tensors holding uint32 values. Returns 4 int64 tensors."""
    c0 = torch.as_tensor(c0, dtype=torch.int64) & MASK32
    c1 = torch.as_tensor(c1, dtype=torch.int64, device=c0.device) & MASK32
    c2 = torch.as_tensor(c2, dtype=torch.int64, device=c0.device) & MASK32
    c3 = torch.as_tensor(c3, dtype=torch.int64, device=c0.device) & MASK32
    c0, c1, c2, c3 = torch.broadcast_tensors(c0, c1, c2, c3)
    k0 &= MASK32
    k1 &= MASK32
    for _ in range(rounds):
        hi0, lo0 = _mulhilo(M0, c0)
        hi1, lo1 = _mulhilo(M1, c2)
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK32, lo1, (hi0 ^ c3 ^ k1) & MASK32, lo0
        k0 = (k0 + W0) & MASK32
        k1 = (k1 + W1) & MASK32
    return c0, c1, c2, c3


def u01_open(u: torch.Tensor) -> torch.Tensor:
    """uint32 -> float64 uniform in (0, 1): 24 high bits, centred.  Matches ``u01_open`` in common.h."""
    return ((u >> 8).to(torch.float64) + 0.5) * (1.0 / 16777216.0)


def seed_key(seed: int):
    s = int(seed) & 0xFFFFFFFFFFFFFFFF
    return s & MASK32, (s >> 32) ^ 0x5EED5EED


def feistel_randperm(n: int, k0: int, k1: int) -> torch.Tensor:
    """Reference of ``randperm_kernel`` (csrc/rl_ops.hip): a 6-round Feistel network on [0, 2^(2h)) with round
    function Philox4x32-10(r, round, 0x5EED, 0; k0, k1).x, cycle-walked until the value is below n.  A bijection of
    [0, n); the kernel's output is bit-identical."""
    bits = 2
    while (1 << bits) < n:
        bits += 1
    h = (bits + 1) // 2
    mask = (1 << h) - 1

    def feistel(x):
        lo, r = x >> h, x & mask
        for rd in range(6):
            f = philox4x32(r, rd, 0x5EED, 0, k0, k1)[0]
            lo, r = r, (lo ^ f) & mask
        return (lo << h) | r

    x = feistel(torch.arange(n, dtype=torch.int64))
    out = x.clone()
    todo = out >= n
    while bool(todo.any()):
        out[todo] = feistel(out[todo])
        todo = out >= n
    return out
