#!/bin/bash
# Kernel stats of a 3-step headline bench (rocprofv3) + the CT phase profile (libmatdcml_ctprof.so, -DMDL_CT_PROF)
# + interleaved training-kernel A/B of every libmatdcml_ab_*.so (flag variants of the current sources).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/kstats.sh || exit 1
bash scripts/ct_prof.sh || exit 2
: > gpurun_out/ct_ab.txt
for round in 1 2; do
for lib in libmatdcml.so $(cd mat_dcml_amd/_lib && ls libmatdcml_ab_*.so 2>/dev/null); do
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 python -u scripts/ct_ab.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ct_ab.txt || exit 3
done
done
