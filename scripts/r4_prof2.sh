#!/bin/bash
# Round-4 profile refresh: CT phase profile, default bench (JSON), every BASELINE config on one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/ct_prof.sh > /dev/null || exit 5
grep -v amdgpu.ids gpurun_out/ct_prof.txt | head -80
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 2; }
tail -1 gpurun_out/bench_default.log | cut -c1-600
bash scripts/configs_bench.sh | cut -c1-400 || exit 6
