"""Evaluate checkpoints on the reference benchmark protocol (DCML_MAT_ALT_Benchmark.py:109-152: AW sweep, 11 points
x 1000 preset decisions, stride 10; the same settings as bench.py's eval block) against the fixed heuristic
(DCML_BID_FIRST_MA_ENV_SingleProcess.py:58-62), and count the sweep points where each checkpoint beats the heuristic
on ct and on payment (BOTH at >= 10 of 11 points).

    python scripts/eval_ckpts.py --n_workers 32 --json out.json ckpt1.pt ckpt2.pt ...
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n_workers", type=int, default=32)
    ap.add_argument("--json", default=None)
    ap.add_argument("--steps", type=int, default=1000, help="decisions per sweep point (the protocol: 1000)")
    ap.add_argument("ckpts", nargs="+")
    a = ap.parse_args()
    from mat_dcml_amd.algos.policy import TransformerPolicy
    from mat_dcml_amd.config import get_config, parse_args
    from mat_dcml_amd.envs.dcml.config import DCMLConfig
    from mat_dcml_amd.envs.dcml.spaces import dcml_action_spaces
    from mat_dcml_amd.runner.benchmark import run_sweep
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    args = parse_args(["--env_name", "DCML", "--n_workers", str(a.n_workers)], get_config(), warn=False)
    cfg = DCMLConfig(n_workers=a.n_workers)
    kw = dict(sweep="AW", n_points=11, steps=a.steps, shards=min(50, a.steps), stride=10, verbose=False, latency_b1=0)
    fixed = run_sweep(None, cfg, dev, fixed=True, **kw)
    out = {"fixed_heuristic": {k: fixed[k] for k in ("ct", "payment", "reward")}, "ckpts": {}}
    print("| checkpoint | ct mean | payment mean | reward mean | ct wins /11 | payment wins /11 | both /11 |")
    print("|---|---|---|---|---|---|---|")
    m = lambda x: sum(x) / len(x)   # noqa: E731
    print(f"| fixed heuristic | {m(fixed['ct']):.4f} | {m(fixed['payment']):.3f} | {m(fixed['reward']):.2f} | | | |")
    for ck in a.ckpts:
        torch.manual_seed(1)
        pol = TransformerPolicy(args, [cfg.obs_dim], [cfg.share_dim], dcml_action_spaces(cfg.n_workers)[0],
                                cfg.n_agents, device=dev)
        pol.restore(ck)
        pol.eval()
        r = run_sweep(pol, cfg, dev, **kw)
        cw = sum(x < y for x, y in zip(r["ct"], fixed["ct"]))
        pw = sum(x < y for x, y in zip(r["payment"], fixed["payment"]))
        bw = sum(x < y and u < v for x, y, u, v in zip(r["ct"], fixed["ct"], r["payment"], fixed["payment"]))
        out["ckpts"][ck] = {"ct": r["ct"], "payment": r["payment"], "reward": r["reward"], "ct_wins": cw,
                            "payment_wins": pw, "both_wins": bw}
        print(f"| {ck} | {m(r['ct']):.4f} | {m(r['payment']):.3f} | {m(r['reward']):.2f} | {cw} | {pw} | {bw} |",
              flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
