"""DCML benchmark sweep (DCML_MAT_ALT_Benchmark.py protocol) and its output format."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from mat_dcml_amd.envs.dcml.config import DCMLConfig
from mat_dcml_amd.runner.benchmark import load_npy, run_sweep, save_npy, sweep_point

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# fixed heuristic, 100 workers, available workers 100 -> 20: (ct, payment) measured on the reference's own code
# ("Eval task time (ct) / payment, fixed heuristic")
REF_FIXED = [(0.804, 47.17), (0.813, 43.94), (0.828, 40.53), (0.866, 37.17), (0.889, 33.46), (0.945, 30.32),
             (1.006, 26.75), (1.082, 23.28), (1.238, 20.01), (1.425, 16.90), (1.887, 13.34)]


def test_fixed_heuristic_sweep_matches_reference_numbers():
    res = run_sweep(None, DCMLConfig(n_workers=100), "cpu", sweep="AW", steps=1000, shards=8, fixed=True,
                    verbose=False)
    ct, pay = np.array(res["ct"]), np.array(res["payment"])
    ref = np.array(REF_FIXED)
    # 1000 episodes per point: sampling noise of the means is ~1%; the preset tasks are the same files
    assert np.all(np.abs(ct / ref[:, 0] - 1) < 0.04), ct
    assert np.all(np.abs(pay / ref[:, 1] - 1) < 0.04), pay
    # fewer available workers: slower and cheaper, as in the reference table
    assert ct[-1] > ct[0] and pay[-1] < pay[0]


def test_shards_replay_the_same_tasks():
    cfg = DCMLConfig(n_workers=16)
    a = run_sweep(None, cfg, "cpu", sweep="R", n_points=3, steps=60, shards=1, fixed=True, verbose=False)
    b = run_sweep(None, cfg, "cpu", sweep="R", n_points=3, steps=60, shards=6, fixed=True, verbose=False)
    # same preset tasks; only the Philox env draws differ between layouts -> close means
    assert np.allclose(a["ct"], b["ct"], rtol=0.25)
    assert sweep_point("AW", 10, 100) == {"disable_rate": 80}
    assert sweep_point("AW", 10, 32) == {"disable_rate": 26}


def test_policy_sweep_and_npy_format(tmp_path):
    from mat_dcml_amd.algos.policy import TransformerPolicy
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.envs.dcml.spaces import dcml_action_spaces
    args = parse_args(["--n_workers", "8"], get_config(), warn=False)
    cfg = DCMLConfig(n_workers=8)
    torch.manual_seed(1)
    pol = TransformerPolicy(args, [7], [cfg.share_dim], dcml_action_spaces(8)[0], 9)
    res = run_sweep(pol, cfg, "cpu", sweep="AW", n_points=4, steps=12, shards=3, stride=10, latency_b1=2,
                    verbose=False)
    assert len(res["ct"]) == 4 and res["decision_ms_b1"] > 0
    p = tmp_path / "x.npy"
    save_npy(str(p), res)
    ct, pay = load_npy(str(p))
    assert ct.shape == (4, 1) and pay.shape == (4, 1)


def test_benchmark_cli(tmp_path):
    out = tmp_path / "o.npy"
    r = subprocess.run([sys.executable, os.path.join(REPO, "DCML_MAT_ALT_Benchmark.py"), "--n_workers", "8",
                        "--bench_steps", "10", "--shards", "2", "--n_points", "3", "--out", str(out),
                        "--policy", "random"], cwd=str(tmp_path), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count("ct:") == 3
    ct, pay = load_npy(str(out))
    assert ct.shape == (3, 1)


def test_frontier_verdict_geometry():
    """a policy point ON the heuristic's ct-payment trade-off is not 'beyond' it; below the
    lower hull of the heuristic points it is; a heuristic point better on both objectives dominates it."""
    from mat_dcml_amd.runner.benchmark import frontier_verdict
    pts = {0.5: (1.0, 10.0), 0.7: (2.0, 6.0), 0.9: (4.0, 5.0)}
    on = frontier_verdict(1.5, 8.0, pts)          # the chord between 0.5 and 0.7
    assert not on["beyond"] and abs(on["margin"]) < 1e-9 and on["dominated_by"] == []
    below = frontier_verdict(1.5, 7.0, pts)
    assert below["beyond"] and abs(below["margin"] - 1.0) < 1e-9
    dom = frontier_verdict(2.5, 6.5, pts)
    assert dom["dominated_by"] == [0.7] and not dom["beyond"]
    fast = frontier_verdict(0.9, 12.0, pts)       # faster than every heuristic setting: no verdict
    assert fast["beyond"] is None and fast["margin"] is None and fast["outside"] == "faster"
    assert fast["dominates"] == []
    fast_cheap = frontier_verdict(0.9, 9.0, pts)  # faster AND cheaper than the fastest setting: a measured dominance
    assert fast_cheap["beyond"] is None and fast_cheap["dominates"] == [0.5]
    slow = frontier_verdict(5.0, 4.0, pts)        # slower than every setting: beyond only if cheaper than the cheapest
    assert slow["beyond"] and abs(slow["margin"] - 1.0) < 1e-9
    from mat_dcml_amd.runner.benchmark import frontier_counts
    c = frontier_counts([on, below, dom, fast, fast_cheap, slow])
    assert c == {"beyond": 2, "not_beyond": 2, "faster_than_frontier": 2, "faster_and_dominating": 1, "points": 6}


def test_eval_report_heldout_and_frontier_cpu():
    """eval_report on the CPU env path (heuristic only, 40 decisions): per-sample results for Sample_1 and a
    held-out set, and the heuristic frontier points at every rho."""
    from mat_dcml_amd.envs.dcml.config import DCMLConfig
    from mat_dcml_amd.runner.benchmark import FRONTIER_RATIOS, eval_report
    rep = eval_report(None, DCMLConfig(n_workers=8), "cpu", samples=(1, 4), steps=40, shards=10, n_points=3)
    assert set(rep["per_sample"]) == {1, 4}
    assert len(rep["per_sample"][4]["fixed"]["ct"]) == 3
    assert [float(r) for r in rep["frontier_points"]] == list(FRONTIER_RATIOS)
    # rho = 0.7 on Sample_1 reproduces the protocol's fixed-heuristic sweep
    assert rep["frontier_points"]["0.7"]["ct"] == [round(x, 4) for x in rep["per_sample"][1]["fixed"]["ct"]]
