"""Evaluate checkpoints on the reference benchmark protocol (DCML_MAT_ALT_Benchmark.py:109-152: AW sweep, 11 points
x 1000 preset decisions, stride 10; the same settings as bench.py's eval block) against the fixed heuristic
(DCML_BID_FIRST_MA_ENV_SingleProcess.py:58-62) on the protocol's preset set Sample_1 AND the nine held-out sets
Sample_2..10 (shipped by the reference, never read by its benchmark), plus the heuristic's ct-payment frontier
(K = floor(rho N), rho = 0.3 .. 1.0) per Sample_1 point.

Checkpoints are SELECTED on the held-out sets only (most held-out points where the checkpoint beats the heuristic
on both objectives, then the held-out mean reward), so the Sample_1 numbers reported for the pick are not the ones
it was chosen on.

    python scripts/eval_ckpts.py --n_workers 32 --json out.json ckpt1.pt ckpt2.pt ...
"""
import argparse
import json
import os
import sys

import numpy as np
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
    from mat_dcml_amd.runner.benchmark import eval_report, frontier_counts
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    args = parse_args(["--env_name", "DCML", "--n_workers", str(a.n_workers)], get_config(), warn=False)
    cfg = DCMLConfig(n_workers=a.n_workers)
    kw = dict(steps=a.steps, shards=min(50, a.steps))
    out = {"ckpts": {}}
    print("| checkpoint | held-out both wins /99 | held-out ct / payment wins /99 | held-out reward | "
          "Sample_1 ct / payment / both wins /11 | Sample_1 beyond heuristic frontier /11 |")
    print("|---|---|---|---|---|---|")
    for ck in a.ckpts:
        torch.manual_seed(1)
        pol = TransformerPolicy(args, [cfg.obs_dim], [cfg.share_dim], dcml_action_spaces(cfg.n_workers)[0],
                                cfg.n_agents, device=dev)
        pol.restore(ck)
        pol.eval()
        rep = eval_report(pol, cfg, dev, **kw)
        h = rep["heldout"]
        held_rew = float(np.mean([np.mean(rep["per_sample"][s]["policy"]["reward"]) for s in h["samples"]]))
        s1 = rep["per_sample"][1]
        fc = frontier_counts(rep["frontier"])
        beyond = fc["beyond"]
        ent = {"heldout_both": sum(h["both_wins_per_sample"]), "heldout_ct": sum(h["ct_wins_per_sample"]),
               "heldout_payment": sum(h["payment_wins_per_sample"]), "heldout_reward": held_rew,
               "sample1": {k: s1[k] for k in ("ct_wins", "payment_wins", "both_wins")}, "frontier_beyond": beyond,
               "frontier_counts": fc, "report": rep}
        out["ckpts"][ck] = ent
        print(f"| {ck} | {ent['heldout_both']} | {ent['heldout_ct']} / {ent['heldout_payment']} | {held_rew:.2f} | "
              f"{s1['ct_wins']} / {s1['payment_wins']} / {s1['both_wins']} | {beyond} "
              f"(+{fc['faster_than_frontier']} faster than every setting) |", flush=True)
    best = max(out["ckpts"], key=lambda k: (out["ckpts"][k]["heldout_both"], out["ckpts"][k]["heldout_reward"]))
    out["selected_on_heldout"] = best
    b = out["ckpts"][best]
    print(f"\nselected on the held-out sets: {best}; its Sample_1 (protocol) wins: ct {b['sample1']['ct_wins']}/11, "
          f"payment {b['sample1']['payment_wins']}/11, both {b['sample1']['both_wins']}/11; beyond the heuristic "
          f"frontier at {b['frontier_beyond']}/11 points")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
