#!/bin/bash
# Decode latency with the VGPR-form MFMA build, forward training-kernel layouts A/B (libmatdcml_ab_*.so), CT profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -v -s --timeout 200 --timeout-method thread -p no:cacheprovider -k "latency or smac or wave_decode_matches" > gpurun_out/pytest_decode3.log 2>&1; rc=$?
grep -E "us per env step|passed|failed|FAILED" gpurun_out/pytest_decode3.log | head -20
[ $rc -eq 0 ] || exit 1
: > gpurun_out/ct_ab.txt
for round in 1 2; do
for lib in libmatdcml.so $(cd mat_dcml_amd/_lib && ls libmatdcml_ab_*.so 2>/dev/null); do
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 python -u scripts/ct_ab.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ct_ab.txt || exit 3
done
done
bash scripts/ct_prof.sh > /dev/null || exit 5
grep -v amdgpu.ids gpurun_out/ct_prof.txt | head -80
bash scripts/configs_bench.sh | cut -c1-400 || exit 6
