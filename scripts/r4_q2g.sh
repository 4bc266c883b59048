#!/bin/bash
# One-wave decode with the cross-attention queries in global memory (32 workers: 2 register weight matrices instead
# of 4): decode tests + latency, default and SMAC bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/configs
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_determinism.py -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_q2g.log 2>&1; rc=$?
grep -E "us per env step|passed|failed|FAILED" gpurun_out/pytest_q2g.log | tail -12
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 2; }
tail -1 gpurun_out/bench_default.log | cut -c1-250
timeout -k 10 300 python -u bench.py --config smac --steps 3 --warmup 1 --no_eval > gpurun_out/configs/smac.log 2>&1 || { tail -20 gpurun_out/configs/smac.log; exit 3; }
tail -1 gpurun_out/configs/smac.log | cut -c1-250
