"""Re-derive the frontier verdicts of stored eval_ckpts.py JSON reports with the round-6 definition
(runner/benchmark.frontier_verdict: only a numeric positive payment margin counts as beyond; points faster than every
heuristic setting get no verdict and are counted apart).  Needs reports that kept their per-point data.

    python scripts/frontier_recount.py profiles/r5_eval/r4_ckpts_heldout.json > profiles/r6_eval/r4_recount.md
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from mat_dcml_amd.runner.benchmark import frontier_counts, frontier_verdict  # noqa: E402


def main(path):
    d = json.load(open(path))
    print("| checkpoint | Sample_1 ct / payment / both wins /11 | beyond (numeric margin > 0) | faster than every "
          "heuristic setting (no verdict) | of those, dominating a heuristic point | behind / on the frontier |")
    print("|---|---|---|---|---|---|")
    for ck, e in d["ckpts"].items():
        rep = e.get("report")
        if rep is None:
            print(f"| {ck} | (no per-point report stored) | | | | |")
            continue
        pol = rep["per_sample"]["1"]["policy"]
        fp = rep["frontier_points"]
        v = [frontier_verdict(pol["ct"][i], pol["payment"][i], {float(r): (fp[r]["ct"][i], fp[r]["payment"][i])
                                                                for r in fp}) for i in range(len(pol["ct"]))]
        c = frontier_counts(v)
        s1 = e["sample1"]
        print(f"| {ck} | {s1['ct_wins']} / {s1['payment_wins']} / {s1['both_wins']} | {c['beyond']} | "
              f"{c['faster_than_frontier']} | {c['faster_and_dominating']} | {c['not_beyond']} |")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
