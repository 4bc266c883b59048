#!/bin/bash
# decode kernel: correctness + determinism tests, phase profile, micro-bench, end-to-end bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_determinism.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_test.log 2>&1 || { tail -30 gpurun_out/ab_test.log; exit 1; }
tail -1 gpurun_out/ab_test.log
MAT_DCML_LIBNAME=libmatdcml_prof.so timeout -k 10 120 python -u scripts/decode_prof.py || exit 2
timeout -k 10 120 python -u -c "
import sys; sys.path.insert(0,'tests')
from bench_decode import run
print('decode us/step L=33:', round(run(256,33,50),1), ' L=101:', round(run(256,101,10),1), ' L=129:', round(run(256,129,10),1))
" || exit 3
timeout -k 10 150 python -u bench.py --steps 4 --warmup 1 --no_eval | tail -1 | cut -c1-200
