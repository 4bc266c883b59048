#!/bin/bash
# A/B of library variants inside the headline bench (rocprofv3 kernel stats of bench.py --steps 3): the training
# kernels as the trainer runs them (32-copy gradient workspace, PPO loss gradients) — the micro-benchmark's absolute
# backward times read ~25 % high.
#   AB_LIBS="libmatdcml.so libmatdcml_ab_x.so" [BENCH_ARGS="--n_workers 100"] bash scripts/r5_benchab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/benchab
export TMPDIR=/tmp
tag=${TAG:-w32}
for lib in ${AB_LIBS:-libmatdcml.so}; do
  d=gpurun_out/benchab/${lib%.so}_$tag
  rm -rf $d
  MAT_DCML_LIBNAME=$lib timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no_eval --no_phase_timers $BENCH_ARGS > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  cp $f $d.kernel_stats.csv
  python3 - "$f" "$lib" "$tag" "$d.log" <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
want = {"mat_enc_fwd_ct<2, true>": "enc_fwd", "mat_dec_fwd_ct<2, true": "dec_fwd", "mat_dec_bwd_ct": "dec_bwd",
        "mat_enc_bwd_ct": "enc_bwd", "decode": "decode"}
out = {}
for r in rows:
    for k, v in want.items():
        if k in r["Name"] and v not in out:
            out[v] = float(r["AverageNs"]) / 1e3
tot = sum(float(r["TotalDurationNs"]) for r in rows) / 4 / 1e6
val = [json.loads(l) for l in open(sys.argv[4]) if l.startswith("{")]
v = val[-1]["value"] if val else 0
print(f"{sys.argv[2]:30s} {sys.argv[3]:5s} " + " ".join(f"{k} {out.get(k, 0):7.1f}" for k in ("enc_fwd", "dec_fwd", "dec_bwd", "enc_bwd", "decode"))
      + f" | four {sum(out.get(k, 0) for k in ('enc_fwd', 'dec_fwd', 'dec_bwd', 'enc_bwd')):7.1f} us | kernels/iter {tot:6.2f} ms | bench {v:9.0f}")
PY
  find $d -name "*kernel_trace.csv" -delete
done | tee -a gpurun_out/benchab/summary.txt
