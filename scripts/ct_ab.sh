#!/bin/bash
# A/B timing of training-kernel variants: every mat_dcml_amd/_lib/libmatdcml_ab_*.so against the default library.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# two interleaved rounds (A B C A B C): the first process on a fresh box runs at lower clocks
for round in 1 2; do
for lib in libmatdcml.so $(cd mat_dcml_amd/_lib && ls libmatdcml_ab_*.so 2>/dev/null); do
  MAT_DCML_LIBNAME=$lib timeout -k 10 120 python -u scripts/ct_ab.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ct_ab.txt || exit 1
done
done
for cp in ${AB_COPIES:-}; do
  MAT_DCML_GRAD_COPIES=$cp timeout -k 10 120 python -u scripts/ct_ab.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ct_ab.txt || exit 1
done
