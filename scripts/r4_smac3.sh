#!/bin/bash
# obs-embedding forward variant check: the SMAC-shaped training test, then SMAC kernel statistics.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "smac or 1288 or od" > gpurun_out/pytest_oe.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" gpurun_out/pytest_oe.log | tail -4
[ $rc -eq 0 ] || exit 1
rm -rf gpurun_out/smacprof
bash scripts/r4_smac_prof.sh
