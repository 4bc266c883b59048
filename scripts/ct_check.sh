#!/bin/bash
# Round-2 CT training kernels: numerics vs fp32 autograd, then bench (CT vs round-1 kernels) and kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_ppo.py tests/test_gpu_rl_ops.py tests/test_dist.py -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ct_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|error|assert" gpurun_out/ct_tests.log | head -40; tail -3 gpurun_out/ct_tests.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no_eval > gpurun_out/bench_ct.log 2>&1 || { tail -20 gpurun_out/bench_ct.log; exit 2; }
grep -o '"value": [0-9.]*' gpurun_out/bench_ct.log
MAT_DCML_TRAIN_KERNELS=v1 timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no_eval > gpurun_out/bench_v1.log 2>&1 || { tail -20 gpurun_out/bench_v1.log; exit 2; }
grep -o '"value": [0-9.]*' gpurun_out/bench_v1.log
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no_eval > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 3; }
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats_ct.csv
find gpurun_out/prof -name "*kernel_trace.csv" -exec rm {} \;
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/kernel_stats_ct.csv")))
for r in rows[:10]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  {int(r["Calls"]):5d} calls  {r["Name"][:70]}')
PY
