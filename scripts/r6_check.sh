#!/bin/bash
# Round-6 check: optional diagnostic script ($DIAG), GPU tests ($TESTS, pytest -k expression over tests/ -m gpu),
# a short bench and rocprofv3 kernel stats ($PROF=1).  Every GPU step under its own time limit, chained.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$DIAG" ]; then
  timeout -k 10 240 python -u $DIAG > gpurun_out/r6_diag_out.txt 2>&1 || { tail -30 gpurun_out/r6_diag_out.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r6_diag_out.txt | tail -20
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -k "$TESTS" -x -v -s --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r6_tests.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|\[perf\]|\[grad-margin\]|\[logprob\]|passed|failed" gpurun_out/r6_tests.log | tail -60
  [ $rc -ne 0 ] && { grep -E "^E " gpurun_out/r6_tests.log | head -30; exit 2; }
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no_eval $BENCH_ARGS > gpurun_out/r6_bench.log 2>&1 || { tail -20 gpurun_out/r6_bench.log; exit 3; }
  tail -1 gpurun_out/r6_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', d['value'], d['ms_per_step'], d.get('phase_ms_per_step'), d.get('train_kernels_ms_per_minibatch'))"
fi
if [ -n "$PROF" ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no_eval --no_phase_timers $BENCH_ARGS > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 4; }
  f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/kernel_stats.csv
  find gpurun_out/prof -name "*kernel_trace.csv" -delete
  python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/kernel_stats.csv")))
for r in rows[:14]:
    print(f"{float(r['AverageNs'])/1e3:9.1f} us x {r['Calls']:>5}  {r['Name'][:110]}")
PY
fi
