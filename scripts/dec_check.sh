#!/bin/bash
# Decode kernel: parity tests, headline bench, per-phase cycle profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_dec.log 2>&1; rc=$?
grep -E "passed|failed|Error|assert" gpurun_out/t_dec.log | tail -n 12; [ $rc = 0 ] || exit 2
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no_eval > gpurun_out/bench_dec.log 2>&1 || { tail -20 gpurun_out/bench_dec.log; exit 3; }
grep -o '"value": [0-9.]*' gpurun_out/bench_dec.log
MAT_DCML_LIBNAME=libmatdcml_prof.so timeout -k 10 200 python -u scripts/decode_prof.py > gpurun_out/decode_prof.txt 2>&1 || exit 4
grep -v amdgpu gpurun_out/decode_prof.txt
