#!/bin/bash
# gradient-test error margins (worst error / limit) of the default build vs the bf16-only self-attention output build
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in libmatdcml.so libmatdcml_ab_olos.so; do
  echo "== $lib"
  MAT_DCML_LIBNAME=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -q -s --timeout 120 --timeout-method thread -p no:cacheprovider -k "grads" > gpurun_out/pytest_margin.log 2>&1
  rc=$?
  grep -E "grad-margin|passed|failed" gpurun_out/pytest_margin.log
  grep -E "attn1.query.bias|attn.query.bias" gpurun_out/pytest_margin.log | head -8
done
