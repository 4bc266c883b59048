#!/bin/bash
# Round-4 one-wave decode check: stage dump (debug library), per-row errors, decode GPU tests (one-wave vs 4-wave vs
# torch, latencies), the headline bench with the one-wave and with the 4-wave decode (MAT_DCML_DECODE_WAVE=0),
# kernel stats, the CT phase profile of the training kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MAT_DCML_LIBNAME=libmatdcml_wdbg.so timeout -k 10 200 python -u scripts/wave_debug.py 2>&1 | grep -v amdgpu.ids | head -30 || exit 1
timeout -k 10 200 python -u scripts/wave_debug.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_decode.log 2>&1; rc=$?
grep -E "us per env step|passed|failed|FAILED" gpurun_out/pytest_decode.log | head -30
[ $rc -eq 0 ] || { grep -B5 "Error" gpurun_out/pytest_decode.log | head -60; exit 2; }
for arm in wave 4wave; do
  [ $arm = 4wave ] && export MAT_DCML_DECODE_WAVE=0 || export MAT_DCML_DECODE_WAVE=1
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no_eval > gpurun_out/bench_$arm.log 2> gpurun_out/bench_$arm.err || { tail -20 gpurun_out/bench_$arm.err; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('phase_ms_per_step'), d.get('train_kernels_ms_per_minibatch'), d.get('kernels',{}).get('decode'))" gpurun_out/bench_$arm.log $arm
done
export MAT_DCML_DECODE_WAVE=1
bash scripts/kstats.sh || exit 4
bash scripts/ct_prof.sh > /dev/null || exit 5
grep -v amdgpu.ids gpurun_out/ct_prof.txt | head -90
