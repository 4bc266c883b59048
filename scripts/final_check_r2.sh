#!/bin/bash
# Round-2 end rehearsal in one GPU call: the round-end checks of scripts/final_check.sh (every GPU test, smoke(),
# default bench with the eval block, rocprofv3 kernel stats), then the decode phase profile of the current kernel
# and a 2-rank bench rehearsal with the auto-probed gradient all-reduce (both ranks on the box's one GPU, gloo).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/final_check.sh || exit $?
MAT_DCML_LIBNAME=libmatdcml_prof.so timeout -k 10 200 python -u scripts/decode_prof.py > gpurun_out/decode_prof.txt 2>&1 || { tail -20 gpurun_out/decode_prof.txt; exit 5; }
grep -v amdgpu gpurun_out/decode_prof.txt | head -16
MAT_DCML_SHARE_DEVICES=1 MAT_DCML_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --allreduce auto --steps 2 --warmup 1 --no_eval > gpurun_out/bench2_auto.log 2>&1 || { tail -30 gpurun_out/bench2_auto.log; exit 6; }
tail -1 gpurun_out/bench2_auto.log | cut -c1-200
grep -o '"grad_allreduce.*' gpurun_out/bench2_auto.log | tail -1
