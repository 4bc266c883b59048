#!/bin/bash
# kernel-time stats of a 3-step bench (rocprofv3 --kernel-trace --stats)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no_eval > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 3; }
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats.csv
find gpurun_out/prof -name "*kernel_trace.csv" -exec rm {} \;
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/kernel_stats.csv")))
for r in rows[:7]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  {int(r["Calls"]):5d} calls  {r["Name"][:70]}')
PY
