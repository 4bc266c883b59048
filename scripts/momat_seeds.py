"""Seed-robust comparison of multi-objective MAT runs with the published MOMAT curves.

    python scripts/momat_seeds.py momat=run_s1.jsonl,run_s2.jsonl,run_s3.jsonl momat_lrdecay=...

For each group: the mean of average_step_objective_{0,1} (= per-step -completion time, -payment;
dcml_runner.py:306-309) over the published run's last window (750k-800k env steps, the last 50 of its 800 logs,
data/dcml_benchmark/momat_{ct,payment}.csv:752-801) per seed, then mean +- sample std over seeds.  Verdict per
objective (both are negated costs: higher is better): "beats" only when the seed mean is above the published window
mean by more than 2 seed std, "worse" when below by more than 2 seed std, otherwise "matches"."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from momat_compare import ours, published, window  # noqa: E402

LO, HI = 750000, 800000


def msd(xs):
    m = sum(xs) / len(xs)
    sd = math.sqrt(sum((x - m) ** 2 for x in xs) / (len(xs) - 1)) if len(xs) > 1 else float("nan")
    return m, sd


def verdict(m, sd, pub):
    if not sd == sd:   # one seed: no claim
        return "n/a (1 seed)"
    if m - pub > 2 * sd:
        return "beats"
    if pub - m > 2 * sd:
        return "worse"
    return "matches"


def main(args):
    pub = {"ct": window(published("ct"), LO, HI), "payment": window(published("payment"), LO, HI)}
    print(f"| group | seeds | objective | per-seed mean {LO // 1000}k-{HI // 1000}k | seed mean +- std | published | "
          f"gap / seed std | verdict |")
    print("|---|---|---|---|---|---|---|---|")
    for arg in args:
        name, _, paths = arg.partition("=")
        paths = [p for p in paths.split(",") if p]
        for obj, key in (("ct", "average_step_objective_0"), ("payment", "average_step_objective_1")):
            per = [window(ours(p, key), LO, HI) for p in paths]
            per = [x for x in per if x == x]
            if not per:
                print(f"| {name} | 0 | {obj} | (no data in the window) ||||||")
                continue
            m, sd = msd(per)
            gap = (m - pub[obj]) / sd if sd and sd == sd else float("nan")
            print(f"| {name} | {len(per)} | {obj} | {', '.join(f'{x:.3f}' for x in per)} | {m:.3f} +- {sd:.3f} | "
                  f"{pub[obj]:.3f} | {gap:+.1f} | {verdict(m, sd, pub[obj])} |")


if __name__ == "__main__":
    main(sys.argv[1:])
