#!/bin/bash
# speculative-block-0 decode: parity tests, latency, then the bench decode kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/perf_guards.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_spec.log 2>&1
rc=$?
grep -E "\[perf\]|passed|failed|Error|assert" gpurun_out/pytest_spec.log | head -40
[ $rc -eq 0 ] || exit $rc
AB_LIBS="libmatdcml.so" bash scripts/r5_benchab.sh || exit 2
d=gpurun_out/benchab/smac; rm -rf $d
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --config smac --steps 3 --warmup 1 --no_eval > $d.log 2>&1 || { tail -5 $d.log; exit 4; }
cp $(find $d -name "*kernel_stats.csv" | head -1) gpurun_out/benchab/smac.kernel_stats.csv; find $d -name "*kernel_trace.csv" -delete
grep '"metric"' $d.log | cut -c1-200
head -4 gpurun_out/benchab/smac.kernel_stats.csv | cut -d, -f1-4
