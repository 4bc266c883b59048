#!/bin/bash
# Training-kernel check: fused-trainer GPU tests (every gradient vs fp32 autograd), determinism, the headline bench,
# kernel stats, then the decode PMC pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_determinism.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_train.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" gpurun_out/pytest_train.log | tail -5
[ $rc -eq 0 ] || { grep -B2 -A12 "Error" gpurun_out/pytest_train.log | head -80; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no_eval > gpurun_out/bench_t.log 2> gpurun_out/bench_t.err || { tail -20 gpurun_out/bench_t.err; exit 3; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('phase_ms_per_step'), d.get('train_kernels_ms_per_minibatch'))" gpurun_out/bench_t.log
bash scripts/kstats.sh || exit 4
[ -n "$SKIP_PMC" ] || bash scripts/decode_pmc2.sh || exit 5
