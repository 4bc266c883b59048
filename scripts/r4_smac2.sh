#!/bin/bash
# Full GPU suite, SMAC bench (8-wave prefetching obs embedding, in-place single minibatch), default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/configs
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_full.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu_full.log | tail -6
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --config smac --steps 3 --warmup 1 --no_eval > gpurun_out/configs/smac.log 2>&1 || { tail -20 gpurun_out/configs/smac.log; exit 2; }
tail -1 gpurun_out/configs/smac.log | cut -c1-250
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 3; }
tail -1 gpurun_out/bench_default.log | cut -c1-250
