#!/bin/bash
# One-shot peer-memory all-reduce on the GPU box: its tests (2 ranks mapping each other's regions over HIP IPC on
# the one GPU) and a 2-rank bench rehearsal whose gradient average runs on the one-shot kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_oneshot.py tests/test_dist.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/oneshot_tests.log 2>&1 || { tail -40 gpurun_out/oneshot_tests.log; exit 1; }
tail -5 gpurun_out/oneshot_tests.log
MAT_DCML_SHARE_DEVICES=1 MAT_DCML_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --allreduce auto --steps 2 --warmup 1 --no_eval > gpurun_out/oneshot_bench2.log 2>&1 || { tail -30 gpurun_out/oneshot_bench2.log; exit 2; }
tail -2 gpurun_out/oneshot_bench2.log
