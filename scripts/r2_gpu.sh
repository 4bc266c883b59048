#!/bin/bash
# Round-2 GPU check: gpu tests, bench (5 timed steps + eval sweep), --gpus 2 on a 1-GPU box must fail loudly
# under RCCL, rocprofv3 kernel stats of a 3-step bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 2; }
tail -1 gpurun_out/bench.log
timeout -k 10 120 python -u bench.py --gpus 2 --steps 1 --warmup 0 --no_eval > gpurun_out/bench_gpus2.log 2>&1; rc=$?
echo "bench --gpus 2 on one GPU: rc=$rc (expected nonzero, not 124)"; grep -m1 "needs one GPU" gpurun_out/bench_gpus2.log
[ $rc -eq 124 ] && exit 4
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no_eval > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 3; }
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats.csv
find gpurun_out/prof -name "*kernel_trace.csv" -exec rm {} \;
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/kernel_stats.csv")))
for r in rows[:8]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  {int(r["Calls"]):5d} calls  {r["Name"][:70]}')
PY
