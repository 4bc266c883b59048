#!/bin/bash
# speculative decode with the token-table rows at L = 101: parity + latency, then the 100-worker bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/perf_guards.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider -k "spec or latency" > gpurun_out/pytest_spec2.log 2>&1
rc=$?
grep -E "\[perf\]|passed|failed|Error|assert" gpurun_out/pytest_spec2.log | head -40
[ $rc -eq 0 ] || exit $rc
AB_LIBS="libmatdcml.so" TAG=w100 BENCH_ARGS="--n_workers 100" bash scripts/r5_benchab.sh || exit 2
AB_LIBS="libmatdcml.so" TAG=w128 BENCH_ARGS="--n_workers 128" bash scripts/r5_benchab.sh || exit 3
