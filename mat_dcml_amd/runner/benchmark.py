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


# ---------------------------------------------------------------------------------------------------- eval analysis
HELDOUT_SAMPLES = tuple(range(2, 11))   # the reference ships Sample_1..10; its benchmark reads only Sample_1
FRONTIER_RATIOS = (0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9, 1.0)


def run_sweep_sample(policy, cfg: DCMLConfig, device, sample: int, **kw):
    """``run_sweep`` on preset set ``Sample_{sample}`` instead of the protocol's Sample_1."""
    import dataclasses
    return run_sweep(policy, dataclasses.replace(cfg, preset_sample=sample), device, **kw)


def heuristic_frontier(cfg: DCMLConfig, device, ratios=FRONTIER_RATIOS, sample: int = 1, **kw):
    """The fixed heuristic's (ct, payment) trade-off at every sweep point: all available workers with
    K = floor(rho N) (``DCML_BID_FIRST_MA_ENV_SingleProcess.py:58-62`` has rho = 0.7) for each rho.
    Returns {rho: run_sweep result}."""
    import dataclasses
    out = {}
    for rho in ratios:
        c = dataclasses.replace(cfg, fixed_k_ratio=float(rho), preset_sample=sample)
        out[float(rho)] = run_sweep(None, c, device, fixed=True, latency_b1=0, **kw)
    return out


def frontier_verdict(ct: float, pay: float, pts) -> dict:
    """Where a policy's (ct, payment) point lies against the heuristic's frontier ``pts`` = [(ct_rho, pay_rho)]:
    * ``dominated_by``: the ratios whose heuristic point is at least as good on both objectives (empty = not
      dominated by any heuristic setting);
    * ``beyond``: the point lies strictly below the lower-left convex hull of the heuristic points in the
      (ct, payment) plane, i.e. no mixture of heuristic settings reaches it — a policy that merely moves along the
      heuristic's trade-off lies ON the curve, not beyond it;
    * ``margin``: payment of the frontier at this ct minus the policy's payment (> 0 = beyond); slower than every
      heuristic point: the cheapest point's payment minus the policy's; None when the policy is FASTER than every
      heuristic point (the frontier is not measured there);
    * ``outside``: "faster" in that last case — then ``beyond`` is None (no verdict: nothing is extrapolated) and
      ``dominates`` lists the heuristic ratios the policy beats on both objectives (a measured comparison).
    Only a numeric positive margin counts as beyond (an unmeasured extrapolation is not evidence)."""
    import numpy as np
    P = sorted((float(c), float(p), r) for r, (c, p) in pts.items())
    dominated = [r for c, p, r in P if c <= ct and p <= pay]
    dominates = [r for c, p, r in P if ct < c and pay < p]
    # lower convex hull (monotone chain), ct ascending
    hull = []
    for c, p, _ in P:
        while len(hull) >= 2 and (hull[-1][0] - hull[-2][0]) * (p - hull[-2][1]) - (hull[-1][1] - hull[-2][1]) * (c - hull[-2][0]) <= 0:
            hull.pop()
        hull.append((c, p))
    xs, ys = np.array([h[0] for h in hull]), np.array([h[1] for h in hull])
    margin, outside = None, None
    if xs[0] <= ct <= xs[-1]:
        margin = float(np.interp(ct, xs, ys) - pay)
    elif ct > xs[-1]:
        margin = float(ys[-1] - pay)   # slower than every heuristic point: beyond only if cheaper than the cheapest
    else:
        outside = "faster"
    beyond = None if margin is None else bool((not dominated) and margin > 0)
    return {"dominated_by": dominated, "dominates": dominates, "beyond": beyond, "outside": outside,
            "margin": None if margin is None else round(margin, 4)}


def frontier_counts(verdicts) -> dict:
    """Summary of ``frontier_verdict`` results: beyond (numeric positive margin), on / behind the frontier, and the
    points faster than every heuristic setting (no verdict) with how many of those still dominate a heuristic point."""
    return {"beyond": sum(v["beyond"] is True for v in verdicts),
            "not_beyond": sum(v["beyond"] is False for v in verdicts),
            "faster_than_frontier": sum(v["outside"] == "faster" for v in verdicts),
            "faster_and_dominating": sum(v["outside"] == "faster" and bool(v["dominates"]) for v in verdicts),
            "points": len(verdicts)}


def eval_report(policy, cfg: DCMLConfig, device, samples=(1,) + HELDOUT_SAMPLES, frontier: bool = True, **kw):
    """The protocol sweep (AW, 11 points x ``steps`` decisions, stride 10) of ``policy`` and of the fixed heuristic
    on every preset set in ``samples``, with per-point wins (policy strictly better on ct / payment / both) and,
    on Sample_1, the heuristic's frontier verdict per point.  ``policy`` None = heuristic only."""
    import numpy as np
    kw = {**dict(sweep="AW", n_points=11, steps=1000, shards=50, stride=10, verbose=False), **kw}
    per = {}
    for s in samples:
        fx = run_sweep_sample(None, cfg, device, s, fixed=True, latency_b1=0, **kw)
        ent = {"fixed": {"ct": fx["ct"], "payment": fx["payment"]}}
        if policy is not None:
            r = run_sweep_sample(policy, cfg, device, s, latency_b1=0, **kw)
            ent["policy"] = {"ct": r["ct"], "payment": r["payment"], "reward": r["reward"]}
            ent["ct_wins"] = int(sum(a < b for a, b in zip(r["ct"], fx["ct"])))
            ent["payment_wins"] = int(sum(a < b for a, b in zip(r["payment"], fx["payment"])))
            ent["both_wins"] = int(sum(a < b and c < d for a, b, c, d in zip(r["ct"], fx["ct"], r["payment"],
                                                                             fx["payment"])))
        per[s] = ent
    out = {"per_sample": per}
    if policy is not None:
        held = [s for s in samples if s != 1]
        def ms(key, field):
            v = np.array([np.mean(per[s]["policy" if field == "p" else "fixed"][key]) for s in held])
            return [round(float(v.mean()), 4), round(float(v.std()), 4)]
        if held:
            out["heldout"] = {"samples": held,
                              "policy_ct_mean_std": ms("ct", "p"), "policy_payment_mean_std": ms("payment", "p"),
                              "fixed_ct_mean_std": ms("ct", "f"), "fixed_payment_mean_std": ms("payment", "f"),
                              "both_wins_per_sample": [per[s]["both_wins"] for s in held],
                              "ct_wins_per_sample": [per[s]["ct_wins"] for s in held],
                              "payment_wins_per_sample": [per[s]["payment_wins"] for s in held]}
    if frontier and 1 in per:
        fr = heuristic_frontier(cfg, device, sample=1, **kw)
        out["frontier_ratios"] = list(fr)
        if policy is not None:
            pol = per[1]["policy"]
            out["frontier"] = [frontier_verdict(pol["ct"][i], pol["payment"][i],
                                                {r: (fr[r]["ct"][i], fr[r]["payment"][i]) for r in fr})
                               for i in range(len(pol["ct"]))]
        out["frontier_points"] = {str(r): {"ct": [round(x, 4) for x in fr[r]["ct"]],
                                           "payment": [round(x, 3) for x in fr[r]["payment"]]} for r in fr}
    return out
