#!/bin/bash
# Decoder training kernels with 3 logit tiles for A <= 48: head-gradient tests (A = 12 / 36 / 60), SMAC kernel stats
# and bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/configs
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ma3.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" gpurun_out/pytest_ma3.log | tail -6
[ $rc -eq 0 ] || exit 1
rm -rf gpurun_out/smacprof
bash scripts/r4_smac_prof.sh > gpurun_out/smacprof_summary.txt || exit 2
head -12 gpurun_out/smacprof_summary.txt
timeout -k 10 300 python -u bench.py --config smac --steps 3 --warmup 1 --no_eval > gpurun_out/configs/smac.log 2>&1 || { tail -20 gpurun_out/configs/smac.log; exit 3; }
tail -1 gpurun_out/configs/smac.log | cut -c1-250
