#!/bin/bash
# Correctness of the current library on the training-kernel GPU tests, then interleaved A/B timing of the training
# kernels (scripts/ct_ab.py) for every mat_dcml_amd/_lib/libmatdcml_ab_*.so against the default library.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest ${AB_TESTS:-tests/test_gpu_train.py} -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ab.log 2>&1 || { tail -40 gpurun_out/pytest_ab.log; exit 1; }
tail -2 gpurun_out/pytest_ab.log
fi
: > gpurun_out/ct_ab.txt
for round in 1 2; do
for lib in libmatdcml.so $(cd mat_dcml_amd/_lib && ls libmatdcml_ab_*.so 2>/dev/null); do
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 python -u scripts/ct_ab.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ct_ab.txt || exit 2
done
done
