#!/bin/bash
# SMAC insert / obs-embedding backward reduction fixes: their tests, then SMAC kernel statistics and bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/configs
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_smac_env.py -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "smac or 1288 or insert" > gpurun_out/pytest_oe.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" gpurun_out/pytest_oe.log | tail -4
[ $rc -eq 0 ] || exit 1
rm -rf gpurun_out/smacprof
bash scripts/r4_smac_prof.sh || exit 2
timeout -k 10 300 python -u bench.py --config smac --steps 3 --warmup 1 --no_eval > gpurun_out/configs/smac.log 2>&1 || { tail -20 gpurun_out/configs/smac.log; exit 3; }
tail -1 gpurun_out/configs/smac.log | cut -c1-250
