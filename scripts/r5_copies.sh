#!/bin/bash
# gradient-workspace copies A/B (MAT_DCML_GRAD_COPIES) in the bench: rocprof kernel stats per setting
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/copies
export TMPDIR=/tmp
for n in 32 64 128 16 32 64; do
  d=gpurun_out/copies/c${n}_$RANDOM
  MAT_DCML_GRAD_COPIES=$n timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no_eval --no_phase_timers > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$n" "$d.log" <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = {}
for r in rows:
    for k, v in {"mat_dec_bwd_ct": "dec_bwd", "mat_enc_bwd_ct": "enc_bwd", "grad_reduce": "reduce"}.items():
        if k in r["Name"] and v not in out:
            out[v] = float(r["AverageNs"]) / 1e3
val = [json.loads(l) for l in open(sys.argv[3]) if l.startswith("{")]
print(f"copies {sys.argv[2]:>4s} " + " ".join(f"{k} {v:7.1f}" for k, v in out.items()) + f" bench {val[-1]['value'] if val else 0:9.0f}")
PY
  find $d -name "*kernel_trace.csv" -delete
done
