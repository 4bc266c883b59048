#!/bin/bash
# Rollout path: decode / insert / determinism GPU tests, headline bench, rocprof kernel stats (launch counts).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_rl_ops.py tests/test_gpu_determinism.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_roll.log 2>&1; rc=$?
grep -E "passed|failed|Error|assert" gpurun_out/t_roll.log | tail -n 12; [ $rc = 0 ] || exit 2
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no_eval > gpurun_out/bench_roll.log 2>&1 || { tail -20 gpurun_out/bench_roll.log; exit 3; }
grep -o '"value": [0-9.]*' gpurun_out/bench_roll.log
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no_eval > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 4; }
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats_roll.csv
find gpurun_out/prof -name "*kernel_trace.csv" -exec rm {} \;
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/kernel_stats_roll.csv")))
print("launches per iteration:", sum(int(r["Calls"]) for r in rows) / 4)
for r in rows[:8]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  {int(r["Calls"]):5d} calls  {r["Name"][:70]}')
PY
