#!/bin/bash
# training kernels: parity + determinism tests, section profile, end-to-end bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_determinism.py tests/test_gpu_ppo.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_test.log 2>&1 || { tail -30 gpurun_out/ab_test.log; exit 1; }
tail -1 gpurun_out/ab_test.log
MAT_DCML_LIBNAME=libmatdcml_tprof.so timeout -k 10 120 python -u scripts/train_prof.py || exit 2
timeout -k 10 150 python -u bench.py --steps 4 --warmup 1 --no_eval | tail -1 | cut -c1-200
