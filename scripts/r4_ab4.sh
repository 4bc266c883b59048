#!/bin/bash
# One-wave decode A/B: first key chunk peeled (default build) vs the plain chunk loop (libmatdcml_ab_nopeel.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -v -s --timeout 200 --timeout-method thread -p no:cacheprovider -k "wave_decode or smac or latency" > gpurun_out/pytest_decode4.log 2>&1; rc=$?
grep -E "us per env step|passed|failed|FAILED" gpurun_out/pytest_decode4.log | head -20
[ $rc -eq 0 ] || exit 1
for round in 1 2; do
for lib in libmatdcml_ab_nopeel.so libmatdcml.so; do
  echo "== $lib"
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_decode.py -s -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "wave_decode_latency or smac" 2>&1 | grep -E "us per env step|passed|failed" || exit 3
done
done
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 2; }
tail -1 gpurun_out/bench_default.log | cut -c1-400
