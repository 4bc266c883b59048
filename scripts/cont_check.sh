#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_ppo.py tests/test_mujoco.py -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cont_tests.log 2>&1; rc=$?
grep -E "FAILED|Error|assert" gpurun_out/cont_tests.log | head -20; tail -2 gpurun_out/cont_tests.log
exit $rc
