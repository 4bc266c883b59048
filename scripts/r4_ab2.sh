#!/bin/bash
# Round-4 kernel iteration check in ONE call: the training / decode GPU tests on the default library, interleaved
# A/B timing of the training kernels (scripts/ct_ab.py) and of the decode (test latency prints) for the default
# library vs every _lib/libmatdcml_ab_*.so, then one short headline bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest ${AB_TESTS:-tests/test_gpu_train.py tests/test_gpu_decode.py} -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ab.log 2>&1 || { tail -40 gpurun_out/pytest_ab.log; exit 1; }
tail -2 gpurun_out/pytest_ab.log
fi
: > gpurun_out/ct_ab.txt
for round in 1 2; do
for lib in libmatdcml.so $(cd mat_dcml_amd/_lib && ls libmatdcml_ab_*.so 2>/dev/null); do
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 python -u scripts/ct_ab.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ct_ab.txt || exit 2
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_decode.py -k "latency or smac" > gpurun_out/decode_ab_$lib.log 2>&1 || { tail -30 gpurun_out/decode_ab_$lib.log; exit 3; }
  echo "$lib decode: $(grep -E 'us per env step' gpurun_out/decode_ab_$lib.log | tr '\n' ' ')" | tee -a gpurun_out/ct_ab.txt
done
done
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no_eval > gpurun_out/bench_ab.log 2> gpurun_out/bench_ab.err || { tail -20 gpurun_out/bench_ab.err; exit 4; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d.get('phase_ms_per_step'), d.get('train_kernels_ms_per_minibatch'))" gpurun_out/bench_ab.log
