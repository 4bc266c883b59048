#!/bin/bash
# Round-4 first GPU check: the GPU tests touched by the round-4 fixes, and the phase-timer overhead A/B of bench.py
# (timers on / off, interleaved twice; the timed ms per step must agree within 1 %).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_oneshot.py tests/test_rollout_groups.py tests/test_build_guard.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r4c1.log 2>&1 || { tail -40 gpurun_out/pytest_r4c1.log; exit 1; }
tail -3 gpurun_out/pytest_r4c1.log
for round in 1 2; do
  for arm in "" "--no_phase_timers"; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no_eval $arm > gpurun_out/bench_ab_${round}${arm}.log 2> gpurun_out/bench_ab_${round}${arm}.err || { tail -20 gpurun_out/bench_ab_${round}${arm}.err; exit 3; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2] or 'timers', d['ms_per_step'], d.get('phase_ms_per_step'), d.get('train_kernels_ms_per_minibatch'), d.get('native_build'))" gpurun_out/bench_ab_${round}${arm}.log "$arm"
  done
done
