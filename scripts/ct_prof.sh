#!/bin/bash
# Phase profile of the CT training kernels (-DMDL_CT_PROF builds; CT_PROF_LIBS lists the libraries to compare).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/ct_prof.txt
for lib in ${CT_PROF_LIBS:-libmatdcml_ctprof.so}; do
  echo "== $lib" >> gpurun_out/ct_prof.txt
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 python -u scripts/ct_prof.py >> gpurun_out/ct_prof.txt 2>&1 || { grep -v amdgpu.ids gpurun_out/ct_prof.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/ct_prof.txt
