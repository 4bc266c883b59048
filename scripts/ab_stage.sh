#!/bin/bash
# A/B: decode inputs staged in LDS vs read from HBM in the agent loop
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_determinism.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_test.log 2>&1 || { tail -30 gpurun_out/ab_test.log; exit 1; }
tail -1 gpurun_out/ab_test.log
for st in 0 1 0 1; do
  MAT_DCML_DECODE_STAGE=$st timeout -k 10 120 python -u -c "
import sys; sys.path.insert(0,'tests')
from bench_decode import run
print('stage=$st decode us/step', round(run(256,33,50),1), ' L=101 B=256:', round(run(256,101,10),1))
" || exit 2
done
MAT_DCML_DECODE_STAGE=0 timeout -k 10 150 python -u bench.py --steps 4 --warmup 1 --no_eval | tail -1 | cut -c1-200
MAT_DCML_DECODE_STAGE=1 timeout -k 10 150 python -u bench.py --steps 4 --warmup 1 --no_eval | tail -1 | cut -c1-200
