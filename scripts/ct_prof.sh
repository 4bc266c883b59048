#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MAT_DCML_LIBNAME=libmatdcml_ctprof.so timeout -k 10 200 python -u scripts/ct_prof.py > gpurun_out/ct_prof.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/ct_prof.txt; exit $rc
