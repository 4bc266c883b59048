#!/bin/bash
# kernel-time stats of the 100-worker config (L = 101), 2 timed steps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof100
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof100 -o run --output-format csv -- python3 bench.py --n_workers 100 --steps 2 --warmup 1 --no_eval > gpurun_out/prof100.log 2>&1 || { tail -20 gpurun_out/prof100.log; exit 3; }
f=$(find gpurun_out/prof100 -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats_w100.csv
find gpurun_out/prof100 -name "*kernel_trace.csv" -exec rm {} \;
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/kernel_stats_w100.csv")))
for r in rows[:8]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  {int(r["Calls"]):5d} calls {float(r["Percentage"]):5.1f}%  {r["Name"][:70]}')
PY
