"""Evaluation sweep of the DCML benchmark ("Batch MAT Decision-Making" eval task time / payment).

Protocol = reference ``DCML_MAT_ALT_Benchmark.py:109-152``: for each sweep point i, a preset env
(``Env(preset=True)``, replaying ``data/dcml_benchmark/Sample_1*``) is modified — available workers
(``modify_preset(disable_rate=8 i)``, 11 points), rows R, columns C or loss probability Pr (10 points, the
commented alternatives at ``:122-125``) — and driven for 1000 steps by the deterministic policy with the batch
decision ``stride`` (10).  The mean task completion time (``info["delay"]``) and payment per point are
written as two consecutive ``np.save`` arrays of shape (points, 1) (``:148-152``).

MI355X design: all sweep points AND ``shards`` contiguous slices of each point's 1000-episode sequence run as
independent envs of ONE batched device env (stacked preset tables, per-env first row), so the whole sweep is
``ceil(1000 / shards)`` batched decisions instead of 11,000 sequential batch-1 calls.  Each env replays
exactly the preset tasks its slice covers; only the env-internal randomness (retries, bid noise) comes from
the Philox streams.  Per-decision latency is reported both for the batched call and for a batch-1 call (the
reference's 28.5-30.7 ms CPU figure).
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from ..envs.dcml.config import DCMLConfig
from ..envs.dcml.data import load_preset
from ..envs.dcml.vec_env import DeviceDCMLEnv

DEFAULT_POINTS = {"AW": 11, "R": 10, "C": 10, "Pr": 10}


def sweep_point(sweep: str, i: int, W: int) -> dict:
    """``modify_preset`` arguments of sweep point i (``DCML_MAT_ALT_Benchmark.py:122-125``).  The AW step of 8
    workers (of 100) scales with the worker count."""
    if sweep == "AW":
        return {"disable_rate": min(W - 1, int(round(8 * i * W / 100.0)))}
    if sweep == "R":
        return {"R": round((i + 1) * (2 ** 20) / 10)}
    if sweep == "C":
        return {"R": 2 ** 19, "C": (i + 1) * (2 ** 10) / 10}
    if sweep == "Pr":
        return {"R": 2 ** 19, "C": 2 ** 9, "Pr": i * 0.1}
    raise ValueError(f"unknown sweep {sweep!r} (AW | R | C | Pr)")


def _stacked_tables(cfg: DCMLConfig, sweep: str, n_points: int):
    m0, p0, d0 = load_preset(cfg)
    ms, ps, ds = [], [], []
    for i in range(n_points):
        m, p, d = m0.copy(), p0.copy(), d0.copy()
        kw = sweep_point(sweep, i, cfg.n_workers)
        if "R" in kw:
            m[:, 0] = kw["R"]
        if "C" in kw:
            m[:, 1] = kw["C"]
        if "disable_rate" in kw:
            d[:] = kw["disable_rate"]
        if "Pr" in kw:
            p[:] = kw["Pr"]
        ms.append(m), ps.append(p), ds.append(d)
    return np.concatenate(ms), np.concatenate(ps), np.concatenate(ds), m0.shape[0]


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def run_sweep(policy, cfg: DCMLConfig, device, sweep: str = "AW", n_points: int | None = None, steps: int = 1000,
              shards: int = 8, stride: int = 10, fixed: bool = False, seed: int = 1, latency_b1: int = 20,
              verbose: bool = True):
    """Returns a dict with per-point mean reward / ct / payment and the decision latencies."""
    device = torch.device(device)
    n_points = n_points or DEFAULT_POINTS[sweep]
    master, prs, dis, rows = _stacked_tables(cfg, sweep, n_points)
    if steps > rows - 1:
        raise ValueError(f"preset holds {rows} episodes; at most {rows - 1} steps per sweep point")
    shards = max(1, min(shards, steps))
    chunk = math.ceil(steps / shards)
    E = n_points * shards
    g = np.repeat(np.arange(n_points), shards)
    s = np.tile(np.arange(shards), n_points)
    start = g * rows + s * chunk
    n_valid = torch.as_tensor(np.clip(steps - s * chunk, 0, chunk), device=device)      # steps each env counts
    env = DeviceDCMLEnv(E, cfg, device=device, seed=seed, fixed=fixed, preset=True)
    env.set_preset_tables(master, prs, dis, start)
    obs, _, ava = env.reset()
    sums = torch.zeros(3, E, dtype=torch.float64, device=device)
    lat = []
    zeros = torch.zeros(E, cfg.n_agents, 1, device=device)
    for t in range(chunk):
        _sync(device)
        t0 = time.perf_counter()
        if fixed or policy is None:
            actions = zeros
        else:
            actions = policy.get_actions(None, obs, ava, deterministic=True, stride=stride)[1]
        _sync(device)
        lat.append(time.perf_counter() - t0)
        obs, _, rew, _, delay, pay, ava = env.step(actions)
        keep = (n_valid > t).double()
        sums += torch.stack([rew.double(), delay.double(), pay.double()]) * keep
    per = (sums.view(3, n_points, shards).sum(-1) / float(steps)).cpu().numpy()
    out = {"sweep": sweep, "points": [sweep_point(sweep, i, cfg.n_workers) for i in range(n_points)],
           "reward": per[0].tolist(), "ct": per[1].tolist(), "payment": per[2].tolist(),
           "batched_envs": E, "decisions": chunk, "stride": stride,
           "decision_ms_batched": 1e3 * float(np.median(lat)) if lat else 0.0}
    if policy is not None and not fixed and latency_b1 > 0:
        e1 = DeviceDCMLEnv(1, cfg, device=device, seed=seed, preset=True)
        o1, _, a1 = e1.reset()
        l1 = []
        for _ in range(latency_b1 + 2):
            _sync(device)
            t0 = time.perf_counter()
            act = policy.get_actions(None, o1, a1, deterministic=True, stride=stride)[1]
            _sync(device)
            l1.append(time.perf_counter() - t0)
            o1, _, _, _, _, _, a1 = e1.step(act)
        out["decision_ms_b1"] = 1e3 * float(np.median(l1[2:]))
    if verbose:
        for i in range(n_points):
            print("reward:", out["reward"][i], "ct:", out["ct"][i], "payment:", out["payment"][i])
    return out


def save_npy(path: str, result: dict):
    """Reference output format (``DCML_MAT_ALT_Benchmark.py:148-152``): two arrays of shape (points, 1)."""
    with open(path, "wb") as f:
        np.save(f, np.array(result["ct"]).reshape(-1, 1))
        np.save(f, np.array(result["payment"]).reshape(-1, 1))


def load_npy(path: str):
    with open(path, "rb") as f:
        return np.load(f), np.load(f)
