#!/bin/bash
# MLP pre-activation saves (MDL_SAVE_PREACT=1): training gradient tests (with margins) on that build, then the
# in-bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
MAT_DCML_LIBNAME=libmatdcml_ab_preact.so timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_preact.log 2>&1
rc=$?
grep -E "grad-margin|passed|failed|Error" gpurun_out/pytest_preact.log | head -20
rm -rf gpurun_out/benchab
AB_LIBS="libmatdcml.so libmatdcml_ab_preact.so libmatdcml.so libmatdcml_ab_preact.so" bash scripts/r5_benchab.sh || exit 2
exit $rc
