#!/bin/bash
# Round-3 check: every GPU test, the default bench, the SMAC bench, kernel stats of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_all.txt 2>&1; rc=$?
tail -4 gpurun_out/gpu_all.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 2; }
grep "^{" gpurun_out/bench.log | cut -c1-300
timeout -k 10 300 python -u bench.py --config smac --steps 5 --warmup 2 > gpurun_out/bench_smac.log 2>&1 || { tail -20 gpurun_out/bench_smac.log; exit 3; }
grep "^{" gpurun_out/bench_smac.log | cut -c1-300
for cfg in dcml smac; do
  rm -rf gpurun_out/prof_$cfg
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$cfg -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_$cfg.log 2>&1) || { tail -20 gpurun_out/prof_$cfg.log; exit 4; }
  f=$(find gpurun_out/prof_$cfg -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/kernel_stats_$cfg.csv
  find gpurun_out/prof_$cfg -name "*kernel_trace.csv" -delete
  python3 - $cfg <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/kernel_stats_{sys.argv[1]}.csv")))
print("==", sys.argv[1])
for r in rows[:10]:
    print(f"{float(r['AverageNs'])/1e3:9.1f} us avg {int(r['Calls']):6d} calls  {r['Name'][:90]}")
PY
done
