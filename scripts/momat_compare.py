"""Compare multi-objective MAT runs (logs/summary.json of DCML_MAT_Train.py --algorithm_name momat|dmomat) with
the published MOMAT TensorBoard exports (data/dcml_benchmark/momat_ct.csv, momat_payment.csv).
Objectives are logged as average_step_objective_{0,1} = mean per-step (-completion time, -payment)
(dcml_runner.py:306-309).  Prints a markdown table: first / final / best / mean over the last 1/16 of the run
(the published last-50-of-800 logs) and the values at 10 / 50 / 100 % of the published 800 k-step run."""
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(HERE, "..", "data", "dcml_benchmark")


def published(name):
    rows = list(csv.DictReader(open(os.path.join(DATA, f"momat_{name}.csv"))))
    return [(int(float(r["Step"])), float(r["Value"])) for r in rows]


def ours(path, key):
    if path.endswith(".jsonl"):   # logs/scalars.jsonl: written as the run goes (a run cut at its time limit)
        rows = [json.loads(line) for line in open(path) if line.strip()]
        return [(int(r["step"]), float(r["value"])) for r in rows
                if r["tag"].endswith(key) or r["tag"].split("/")[-1] == key]
    d = json.load(open(path))
    for k, v in d.items():
        if k.endswith(key) or k.split("/")[-1] == key:
            return [(int(s), float(x)) for _, s, x in v]
    return []


def stats(series):
    vals = [v for _, v in series]
    n = max(1, len(vals) // 16)
    return {"first": vals[0], "final": vals[-1], "best": max(vals), "tail_mean": sum(vals[-n:]) / n,
            "steps": series[-1][0], "logs": len(vals)}


def window(series, lo, hi):
    vals = [v for s, v in series if lo <= s <= hi]
    return sum(vals) / len(vals) if vals else float("nan")


def at(series, step):
    best = min(series, key=lambda sv: abs(sv[0] - step))
    return best[1]


def main(paths):
    pub = {"ct": published("ct"), "payment": published("payment")}
    print("| run | objective | env steps (logs) | first | final | best | last-1/16 mean | @80k | @400k | @800k | "
          "mean 750k-800k | mean 400k-800k |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for name, ser in pub.items():
        s = stats(ser)
        print(f"| published MOMAT | {name} | {s['steps']} ({s['logs']}) | {s['first']:.3f} | {s['final']:.3f} | "
              f"{s['best']:.3f} | {s['tail_mean']:.3f} | {at(ser, 80000):.3f} | {at(ser, 400000):.3f} | "
              f"{at(ser, 800000):.3f} | {window(ser, 750000, 800000):.3f} | {window(ser, 400000, 800000):.3f} |")
    for p in paths:
        run = os.path.basename(p).replace("summary_", "").replace(".json", "")
        for name, key in (("ct", "average_step_objective_0"), ("payment", "average_step_objective_1")):
            ser = ours(p, key)
            if not ser:
                print(f"| {run} | {name} | (no {key} in {p}) |||||||")
                continue
            s = stats(ser)
            print(f"| {run} | {name} | {s['steps']} ({s['logs']}) | {s['first']:.3f} | {s['final']:.3f} | "
                  f"{s['best']:.3f} | {s['tail_mean']:.3f} | {at(ser, 80000):.3f} | {at(ser, 400000):.3f} | "
                  f"{at(ser, 800000):.3f} | {window(ser, 750000, 800000):.3f} | {window(ser, 400000, 800000):.3f} |")


if __name__ == "__main__":
    main(sys.argv[1:])
