#!/bin/bash
# perf guards (the tests' own timing, printed + gpurun_out/perf_guards.jsonl), forward-order A/B, configs + kernel
# stats at 100 / 128 workers and SMAC.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/perf_guards.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_decode.py -x -q -s -k "time_bound or latency" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_perf.log 2>&1 || { tail -20 gpurun_out/pytest_perf.log; exit 1; }
grep "\[perf\]" gpurun_out/pytest_perf.log
AB_LIBS="libmatdcml_ab_prev.so libmatdcml.so" bash scripts/r5_benchab.sh || exit 2
for w in 100 128; do
  AB_LIBS="libmatdcml.so" TAG=w$w BENCH_ARGS="--n_workers $w" bash scripts/r5_benchab.sh || exit 3
done
d=gpurun_out/benchab/smac; rm -rf $d
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --config smac --steps 3 --warmup 1 --no_eval > $d.log 2>&1 || { tail -5 $d.log; exit 4; }
cp $(find $d -name "*kernel_stats.csv" | head -1) gpurun_out/benchab/smac.kernel_stats.csv; find $d -name "*kernel_trace.csv" -delete
tail -1 $d.log | cut -c1-200
