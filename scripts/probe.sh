#!/bin/bash
# One GPU call for a training-kernel investigation: GPU tests, bench, kernel stats, then the A/B timing of every
# _lib/libmatdcml_ab_*.so and the phase profile of _lib/libmatdcml_ctprof.so (SKIP_TESTS=1 skips the tests).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no_eval > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 2; }
tail -1 gpurun_out/bench.log | cut -c1-400
bash scripts/kstats.sh || exit 3
rm -f gpurun_out/ct_ab.txt
bash scripts/ct_ab.sh || exit 4
if [ -f mat_dcml_amd/_lib/libmatdcml_ctprof.so ]; then bash scripts/ct_prof.sh > /dev/null || exit 5; cat gpurun_out/ct_prof.txt | head -80; fi
if [ -f mat_dcml_amd/_lib/libmatdcml_prof.so ]; then
  MAT_DCML_LIBNAME=libmatdcml_prof.so timeout -k 10 200 python -u scripts/decode_prof.py > gpurun_out/decode_prof.txt 2>&1 || { tail -20 gpurun_out/decode_prof.txt; exit 6; }
  grep -v amdgpu gpurun_out/decode_prof.txt | head -16
fi
