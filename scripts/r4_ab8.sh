#!/bin/bash
# Register-pressure trackers A/B: on the backward TUs (libmatdcml_ab_bwdtr.so: adds the encoder backward) and on
# every TU (libmatdcml_ab_alltr.so: measured here for the decode kernels).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ct_ab.txt
for round in 1 2; do
for lib in libmatdcml.so libmatdcml_ab_bwdtr.so; do
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 python -u scripts/ct_ab.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ct_ab.txt || exit 3
done
done
for lib in libmatdcml.so libmatdcml_ab_alltr.so libmatdcml.so libmatdcml_ab_alltr.so; do
  echo "== $lib"
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_decode.py -s -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "wave_decode_latency or smac" 2>&1 | grep -E "us per env step|passed|failed" || exit 4
done
