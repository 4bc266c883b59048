#!/bin/bash
# Decode A/B: the decode GPU tests (latency prints) for the default library and every _lib/libmatdcml_ab_*.so,
# two interleaved rounds, then the phase profile of the default build (libmatdcml_prof.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for round in 1 2; do
for lib in libmatdcml.so $(cd mat_dcml_amd/_lib && ls libmatdcml_ab_*.so 2>/dev/null); do
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_decode.py > gpurun_out/decode_ab_$lib.log 2>&1 || { tail -30 gpurun_out/decode_ab_$lib.log; exit 1; }
  echo "$lib: $(grep -E 'us per env step' gpurun_out/decode_ab_$lib.log | tr '\n' ' ') $(tail -1 gpurun_out/decode_ab_$lib.log)"
done
done
MAT_DCML_LIBNAME=libmatdcml_prof.so timeout -k 10 120 python -u scripts/decode_prof.py 2>&1 | grep -v amdgpu.ids > gpurun_out/decode_prof.txt || exit 2
grep -E "cycles total" gpurun_out/decode_prof.txt
