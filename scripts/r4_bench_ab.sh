#!/bin/bash
# Headline bench with the one-wave and the 4-wave decode (MAT_DCML_DECODE_WAVE=0), kernel stats, CT phase profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for arm in wave 4wave wave; do
  [ $arm = 4wave ] && export MAT_DCML_DECODE_WAVE=0 || export MAT_DCML_DECODE_WAVE=1
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no_eval > gpurun_out/bench_$arm.log 2> gpurun_out/bench_$arm.err || { tail -20 gpurun_out/bench_$arm.err; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('phase_ms_per_step'), d.get('train_kernels_ms_per_minibatch'), d.get('kernels',{}).get('decode'))" gpurun_out/bench_$arm.log $arm
done
export MAT_DCML_DECODE_WAVE=1
bash scripts/kstats.sh || exit 4
bash scripts/ct_prof.sh > /dev/null || exit 5
grep -v amdgpu.ids gpurun_out/ct_prof.txt | head -90
