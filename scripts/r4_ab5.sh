#!/bin/bash
# Training kernels A/B: packed LayerNorm backward / delta (default build) vs HEAD~ (libmatdcml_ab_base.so); gradient
# tests; phase profile; bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_train5.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_train5.log | tail -8
[ $rc -eq 0 ] || exit 1
: > gpurun_out/ct_ab.txt
for round in 1 2 3; do
for lib in libmatdcml_ab_base.so libmatdcml.so; do
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 python -u scripts/ct_ab.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ct_ab.txt || exit 3
done
done
bash scripts/ct_prof.sh > /dev/null || exit 5
grep -v amdgpu.ids gpurun_out/ct_prof.txt | head -60
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 2; }
tail -1 gpurun_out/bench_default.log | cut -c1-300
