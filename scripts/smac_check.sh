#!/bin/bash
# SMAC-shaped config (#5) on the fused HIP path: parity tests, bench, kernel stats of the update.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_ppo.py tests/test_gpu_rl_ops.py tests/test_gpu_decode.py tests/test_gpu_smac_env.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/smac_tests.log 2>&1; rc=$?
grep -E "FAILED|Error|assert" gpurun_out/smac_tests.log | head -20; tail -2 gpurun_out/smac_tests.log
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u bench.py --config smac --steps 3 --warmup 1 > gpurun_out/bench_smac.log 2>&1 || { tail -20 gpurun_out/bench_smac.log; exit 2; }
grep -v amdgpu.ids gpurun_out/bench_smac.log | tail -1
rm -rf gpurun_out/prof_smac
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_smac -o run --output-format csv -- python3 bench.py --config smac --steps 2 --warmup 1 > gpurun_out/prof_smac.log 2>&1 || { tail -20 gpurun_out/prof_smac.log; exit 3; }
f=$(find gpurun_out/prof_smac -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats_smac.csv
find gpurun_out/prof_smac -name "*kernel_trace.csv" -exec rm {} \;
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/kernel_stats_smac.csv")))
for r in rows[:14]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us avg  {int(r["Calls"]):5d} calls {float(r["Percentage"]):5.1f}%  {r["Name"][:60]}')
print("GEMM library kernels:", [r["Name"][:50] for r in rows if "Cijk" in r["Name"] or "gemm" in r["Name"].lower()])
PY
