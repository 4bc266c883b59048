#!/bin/bash
# A/B of library variants: fused-training numerics on each variant, then the headline bench for each
# (AB_LIBS lists the libraries; the first is the default build).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/ab_bench.txt
for lib in ${AB_LIBS:-libmatdcml.so}; do
  MAT_DCML_LIBNAME=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_ppo.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests_$lib.log 2>&1 || { echo "$lib tests FAILED"; tail -30 gpurun_out/ab_tests_$lib.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/ab_tests_$lib.log)" | tee -a gpurun_out/ab_bench.txt
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no_eval > gpurun_out/ab_bench_$lib.log 2>&1 || { tail -20 gpurun_out/ab_bench_$lib.log; exit 2; }
  echo "$lib $(grep -o '"value": [0-9.]*' gpurun_out/ab_bench_$lib.log)" | tee -a gpurun_out/ab_bench.txt
done
