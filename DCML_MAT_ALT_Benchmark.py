#!/usr/bin/env python
"""DCML evaluation benchmark (CLI-compatible with the reference ``DCML_MAT_ALT_Benchmark.py``).

Default argv = the reference's hard-coded list (``DCML_MAT_ALT_Benchmark.py:80``): restore
``./results/DCML/AS/mat/check/run1/models/transformer_1900.pt``, decide deterministically with stride 10, sweep
the available workers 100 → 20 over 11 points of 1000 preset episodes each, print one
``reward: … ct: … payment: …`` line per point and write ``dcml_BMAT_RUN1_1900_AW.npy``.

Extra flags: ``--sweep AW|R|C|Pr``, ``--n_points``, ``--bench_steps`` (1000), ``--shards`` (slices of each point
run as parallel envs), ``--stride`` (10), ``--policy mat|fixed|random``, ``--out``, ``--json``,
``--n_workers``.  A missing checkpoint falls back to random-init weights (``torch.manual_seed(seed)``) with a
warning; the reference raises instead.
"""
import argparse
import json
import os
import re
import sys

import numpy as np
import torch

from mat_dcml_amd.config import get_config, parse_args
from mat_dcml_amd.envs.dcml.config import DCMLConfig
from mat_dcml_amd.envs.dcml.spaces import dcml_action_spaces
from mat_dcml_amd.runner.benchmark import run_sweep, save_npy

DEFAULT_ARGV = ["--use_eval", "--n_eval_rollout_threads", "2", "--algorithm_name", "mat", "--model_dir",
                "./results/DCML/AS/mat/check/run1/models/transformer_1900.pt"]


def bench_parser():
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--sweep", default="AW", choices=["AW", "R", "C", "Pr"])
    p.add_argument("--n_points", type=int, default=None)
    p.add_argument("--bench_steps", type=int, default=1000)
    p.add_argument("--shards", type=int, default=8)
    p.add_argument("--stride", type=int, default=10)
    p.add_argument("--policy", default="mat", choices=["mat", "fixed", "random"])
    p.add_argument("--out", default=None)
    p.add_argument("--json", default=None)
    return p


def default_out(model_dir, sweep, policy):
    if policy != "mat":
        return f"dcml_{policy.upper()}_{sweep}.npy"
    m = re.search(r"run(\d+)/models/transformer_(\d+)\.pt$", str(model_dir or ""))
    return f"dcml_BMAT_RUN{m.group(1)}_{m.group(2)}_{sweep}.npy" if m else f"dcml_BMAT_{sweep}.npy"


def main(argv):
    b, rest = bench_parser().parse_known_args(argv)
    all_args = parse_args(rest, get_config(), warn=False)
    device = torch.device("cuda:0" if all_args.cuda and torch.cuda.is_available() else "cpu")
    print("choose to use gpu..." if device.type == "cuda" else "choose to use cpu...")
    torch.set_num_threads(all_args.n_training_threads)
    cfg = DCMLConfig(n_workers=all_args.n_workers, shannon=all_args.shannon)
    torch.manual_seed(all_args.seed)
    np.random.seed(all_args.seed)
    policy = None
    if b.policy == "mat":
        from mat_dcml_amd.algos.policy import TransformerPolicy
        space = dcml_action_spaces(cfg.n_workers)[0]
        policy = TransformerPolicy(all_args, [cfg.obs_dim], [cfg.share_dim], space, cfg.n_agents, device=device)
        if all_args.model_dir and os.path.exists(all_args.model_dir):
            policy.restore(all_args.model_dir)
        else:
            print(f"[benchmark] checkpoint {all_args.model_dir} not found: using random-init weights "
                  f"(torch seed {all_args.seed})", file=sys.stderr)
        policy.eval()
    elif b.policy == "random":
        from mat_dcml_amd.algos.random_policy import RandomPolicy
        policy = RandomPolicy(all_args, None, None, dcml_action_spaces(cfg.n_workers)[0], cfg.n_agents, device)
    res = run_sweep(policy, cfg, device, sweep=b.sweep, n_points=b.n_points, steps=b.bench_steps, shards=b.shards,
                    stride=b.stride, fixed=b.policy == "fixed", seed=all_args.seed)
    out = b.out or default_out(all_args.model_dir, b.sweep, b.policy)
    save_npy(out, res)
    print(f"decision latency: {res['decision_ms_batched']:.3f} ms per batched call ({res['batched_envs']} envs)"
          + (f", {res['decision_ms_b1']:.3f} ms at batch 1" if "decision_ms_b1" in res else ""))
    if b.json:
        with open(b.json, "w") as f:
            json.dump(res, f, indent=1)
    return res


if __name__ == "__main__":
    main(DEFAULT_ARGV + sys.argv[1:])
