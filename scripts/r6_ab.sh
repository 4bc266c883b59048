#!/bin/bash
# Round-6 A/B of the gradient workspace flush (tests/bench_train_kernels.py, hipEvent per kernel) and the bench.
#   AB_LIBS="libmatdcml.so libmatdcml_ab_pf1.so ..."  AB_BENCH="atomic private"
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6_ab
export TMPDIR=/tmp
for lib in ${AB_LIBS:-libmatdcml.so}; do
  for mode in ${AB_MODES:-private}; do
    MAT_DCML_LIBNAME=$lib MAT_DCML_GRAD_MODE=$mode timeout -k 10 120 python -u tests/bench_train_kernels.py 3200 33 20 \
      > gpurun_out/r6_ab/k_${lib}_${mode}.txt 2>&1 || { tail -5 gpurun_out/r6_ab/k_${lib}_${mode}.txt; exit 1; }
    echo "$lib $mode: $(tail -1 gpurun_out/r6_ab/k_${lib}_${mode}.txt)"
  done
done
for mode in ${AB_BENCH:-}; do
  MAT_DCML_GRAD_MODE=$mode timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no_eval > gpurun_out/r6_ab/bench_$mode.log 2>&1 || { tail -5 gpurun_out/r6_ab/bench_$mode.log; exit 2; }
  tail -1 gpurun_out/r6_ab/bench_$mode.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $mode', d['value'], d['ms_per_step'], d.get('phase_ms_per_step'), d.get('train_kernels_ms_per_minibatch'))"
done
