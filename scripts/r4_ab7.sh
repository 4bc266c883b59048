#!/bin/bash
# Forward training kernels A/B: default (2 workgroups per CU) vs one workgroup per CU (512 registers, no spills) vs
# the register-pressure trackers.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ct_ab.txt
for round in 1 2; do
for lib in libmatdcml.so libmatdcml_ab_fwdw1.so libmatdcml_ab_fwdtr.so; do
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 python -u scripts/ct_ab.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ct_ab.txt || exit 3
done
done
