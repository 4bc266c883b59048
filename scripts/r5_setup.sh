#!/bin/bash
# batched weight fill of the speculative decode's setup: decode parity tests, then decode time A/B vs HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_setup.log 2>&1 || { tail -20 gpurun_out/pytest_setup.log; exit 1; }
tail -1 gpurun_out/pytest_setup.log
for lib in libmatdcml_ab_base.so libmatdcml.so libmatdcml_ab_base.so libmatdcml.so; do
  echo "== $lib"
  MAT_DCML_LIBNAME=$lib timeout -k 10 120 python scripts/decode_time.py 2>&1 | grep "decode\]" || exit 2
done
