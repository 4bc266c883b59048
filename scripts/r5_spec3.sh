#!/bin/bash
# staged block-1 q/k/v in the speculative decode: decode tests, then the bench A/B (previous spec build vs this one)
# and SMAC
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/perf_guards.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_spec3.log 2>&1
rc=$?
grep -E "\[perf\]|passed|failed|Error|assert" gpurun_out/pytest_spec3.log | head -40
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/benchab
AB_LIBS="libmatdcml_ab_spec1.so libmatdcml.so" bash scripts/r5_benchab.sh || exit 2
d=gpurun_out/benchab/smac
timeout -k 10 400 python3 bench.py --config smac --steps 3 --warmup 1 --no_eval > $d.log 2>&1 || { tail -5 $d.log; exit 4; }
grep '"metric"' $d.log | cut -c1-200
