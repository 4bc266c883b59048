"""DCML data: worker workload profiles and preset evaluation episodes.

* ``workloads.txt`` holds 100 sequential ``np.save`` records of (20,) float64 background-load fractions,
  read one per worker by the reference (``DCML_BID_FIRST_MA_ENV_SingleProcess.py:33-37``).
* ``dcml_benchmark/Sample_{k}master_states.npy`` = (1001, 3) rows of (R, C, Pr) and
  ``Sample_{k}worker_states.npy`` = (1001, W) worker Prs followed by (1001,) disable counts
  (``:25-31``, ``:174-178``, ``:191-194``).
All files are read with ``allow_pickle=False``.
For W > 100 workers a synthetic generator samples profiles from the empirical level distribution of the
100 real ones with the same "at most 2 consecutive fully-busy slots" property, so
the timeslot loop stays short.
"""
from __future__ import annotations

import os

import numpy as np

from .config import DCMLConfig


def load_profiles(cfg: DCMLConfig) -> np.ndarray:
    """(W, period) float64 base workload profiles."""
    real = []
    if os.path.exists(cfg.workload_file):
        with open(cfg.workload_file, "rb") as f:
            for _ in range(100):
                try:
                    real.append(np.load(f, allow_pickle=False).astype(np.float64))
                except Exception:
                    break
    real = np.stack(real) if real else synthetic_profiles(100, cfg.period, seed=0)
    if cfg.n_workers <= real.shape[0]:
        return np.ascontiguousarray(real[: cfg.n_workers, : cfg.period])
    extra = synthetic_profiles(cfg.n_workers - real.shape[0], cfg.period, seed=1234, like=real)
    return np.ascontiguousarray(np.concatenate([real[:, : cfg.period], extra], 0))


def synthetic_profiles(n: int, period: int, seed: int = 0, like: np.ndarray | None = None) -> np.ndarray:
    rng = np.random.default_rng(seed)
    if like is not None:
        levels, counts = np.unique(np.round(like.reshape(-1), 4), return_counts=True)
        probs = counts / counts.sum()
    else:
        levels = np.array([0.0, 0.15, 0.35, 0.6, 0.85, 1.0])
        probs = np.array([0.05, 0.35, 0.2, 0.15, 0.1, 0.15])
    out = rng.choice(levels, size=(n, period), p=probs)
    # at most two consecutive (cyclic) fully-busy slots
    for i in range(n):
        for t in range(period):
            if out[i, t] >= 1.0 and out[i, t - 1] >= 1.0 and out[i, t - 2] >= 1.0:
                out[i, t] = 0.6
    return out.astype(np.float64)


def load_preset(cfg: DCMLConfig, sample: int | None = None):
    """Returns (master (R,3) float64, worker_prs (R,W) float64, disable (R,) int64)."""
    k = cfg.preset_sample if sample is None else sample
    mpath = os.path.join(cfg.preset_dir, f"Sample_{k}master_states.npy")
    wpath = os.path.join(cfg.preset_dir, f"Sample_{k}worker_states.npy")
    with open(mpath, "rb") as f:
        master = np.load(f, allow_pickle=False).astype(np.float64)
    with open(wpath, "rb") as f:
        prs = np.load(f, allow_pickle=False).astype(np.float64)
        disable = np.load(f, allow_pickle=False).astype(np.int64)
    W = cfg.n_workers
    if prs.shape[1] != W:
        # worker-count generalisation: tile / truncate the recorded Prs, rescale the disable count
        reps = int(np.ceil(W / prs.shape[1]))
        prs = np.tile(prs, (1, reps))[:, :W]
        disable = np.clip(np.round(disable * W / 100.0).astype(np.int64), 0, W - 1)
    return master, np.ascontiguousarray(prs), disable


def save_preset(path_prefix: str, master: np.ndarray, worker_prs: np.ndarray, disable: np.ndarray):
    """Write a preset in the reference format (``generate_preset_data``, ENV_SingleProcess.py:316-343)."""
    with open(path_prefix + "master_states.npy", "wb") as f:
        np.save(f, np.asarray(master, dtype=np.float64))
    with open(path_prefix + "worker_states.npy", "wb") as f:
        np.save(f, np.asarray(worker_prs, dtype=np.float64))
        np.save(f, np.asarray(disable, dtype=np.int64))
