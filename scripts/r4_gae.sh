#!/bin/bash
# GAE scan with 8-step load prefetch: rl_ops GPU tests, SMAC and default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/configs
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rl_ops.py tests/test_gpu_determinism.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gae.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" gpurun_out/pytest_gae.log | tail -4
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --config smac --steps 3 --warmup 1 --no_eval > gpurun_out/configs/smac.log 2>&1 || { tail -20 gpurun_out/configs/smac.log; exit 3; }
tail -1 gpurun_out/configs/smac.log | cut -c1-250
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 4; }
tail -1 gpurun_out/bench_default.log | cut -c1-250
