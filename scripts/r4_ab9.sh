#!/bin/bash
# Per-file flags A/B on the training kernels: default (trackers on the decoder backward and encoder forward units)
# vs no per-file flags (libmatdcml_ab_noper.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ct_ab.txt
for round in 1 2 3; do
for lib in libmatdcml.so libmatdcml_ab_noper.so; do
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 python -u scripts/ct_ab.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ct_ab.txt || exit 3
done
done
