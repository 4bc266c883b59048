#!/bin/bash
# attention output saved as bf16 only (MDL_SAVE_OLO=0): the training-kernel gradient tests on that build, then the
# in-bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
MAT_DCML_LIBNAME=libmatdcml_ab_olos.so timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_olos.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_olos.log
rm -rf gpurun_out/benchab
AB_LIBS="libmatdcml.so libmatdcml_ab_olos.so libmatdcml.so libmatdcml_ab_olos.so" bash scripts/r5_benchab.sh || exit 2
exit $rc
