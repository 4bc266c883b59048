#!/bin/bash
# Decode with 3 logit tiles for A <= 48 (SMAC): decode tests, then the SMAC bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/configs
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dec5.log 2>&1; rc=$?
grep -E "us per env step|passed|failed|FAILED" gpurun_out/pytest_dec5.log | tail -12
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --config smac --steps 3 --warmup 1 --no_eval > gpurun_out/configs/smac.log 2>&1 || { tail -20 gpurun_out/configs/smac.log; exit 3; }
tail -1 gpurun_out/configs/smac.log | cut -c1-250
