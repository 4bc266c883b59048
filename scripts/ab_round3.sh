#!/bin/bash
# Round-3 A/B: decode tests (wide head) + phase profile, grouped rollout GPU test, 12-wave backward variant + hipEvent
# A/B, bench with 1 vs 2 rollout groups.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/ct_ab.txt
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_decode.py > gpurun_out/decode_tests.log 2>&1 || { tail -40 gpurun_out/decode_tests.log; exit 1; }
grep -E "us per env step|passed|failed" gpurun_out/decode_tests.log
MAT_DCML_LIBNAME=libmatdcml_prof.so timeout -k 10 120 python -u scripts/decode_prof.py > gpurun_out/decode_prof.txt 2>&1 || { tail -20 gpurun_out/decode_prof.txt; exit 1; }
grep -E "cycles total|J head" gpurun_out/decode_prof.txt
timeout -k 10 200 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_rollout_groups.py -m gpu > gpurun_out/groups_test.log 2>&1 || { tail -30 gpurun_out/groups_test.log; exit 1; }
grep -E "rollout_groups=|passed|failed" gpurun_out/groups_test.log
if [ -f mat_dcml_amd/_lib/libmatdcml_ab_w12.so ]; then
  MAT_DCML_LIBNAME=libmatdcml_ab_w12.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py > gpurun_out/w12_tests.log 2>&1; tail -2 gpurun_out/w12_tests.log
fi
bash scripts/ct_ab.sh || exit 1
for g in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no_eval --rollout_groups $g > gpurun_out/bench_g$g.log 2>&1 || { tail -20 gpurun_out/bench_g$g.log; exit 2; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_g$g.log').read().strip().splitlines()[-1]); print('groups', $g, d['value'], d['ms_per_step'])"
done
timeout -k 10 200 python -u bench.py --config smac --steps 3 --warmup 1 > gpurun_out/bench_smac.log 2>&1 || { tail -20 gpurun_out/bench_smac.log; exit 3; }
tail -1 gpurun_out/bench_smac.log | cut -c1-200
