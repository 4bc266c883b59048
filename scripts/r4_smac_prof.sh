#!/bin/bash
# Kernel statistics of the SMAC-shaped config (rocprofv3 --kernel-trace --stats).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/smacprof -o run -- python3 bench.py --config smac --steps 3 --warmup 1 --no_eval > gpurun_out/smacprof.log 2>&1 || { tail -20 gpurun_out/smacprof.log; exit 1; }
tail -1 gpurun_out/smacprof.log | cut -c1-200
f=$(find gpurun_out/smacprof -name "*kernel_stats.csv" | head -1)
cp $f gpurun_out/smac_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/smac_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total ms", tot / 1e6)
for r in rows[:25]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:9.1f}us {float(r['TotalDurationNs'])/1e6:8.2f}ms")
PY
