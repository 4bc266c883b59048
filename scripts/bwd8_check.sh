#!/bin/bash
# 8-wave backward CT kernels: fused-training numerics vs fp32 autograd, then A/B kernel timing vs the 4-wave build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_ppo.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/bwd8_tests.log 2>&1; rc=$?
tail -3 gpurun_out/bwd8_tests.log
grep -E "FAILED|Error" gpurun_out/bwd8_tests.log | head -5
[ $rc -ne 0 ] && exit 1
rm -f gpurun_out/ct_ab.txt
bash scripts/ct_ab.sh
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no_eval > gpurun_out/bench_bwd8.log 2>&1 || { tail -20 gpurun_out/bench_bwd8.log; exit 2; }
grep -o '"value": [0-9.]*' gpurun_out/bench_bwd8.log
