#!/bin/bash
# A/B of compiler-flag library variants (libmatdcml_ab_*.so) on the whole bench: wall-clock env-steps/s and the
# rocprofv3 per-kernel averages of the hot kernels, one library per process (MAT_DCML_LIBNAME).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abf
export TMPDIR=/tmp
for lib in libmatdcml.so $(cd mat_dcml_amd/_lib && ls libmatdcml_ab_*.so 2>/dev/null); do
  echo "== $lib"
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no_eval 2>/dev/null | tail -1 | grep -o '"value": [0-9.]*' || exit 1
  rm -rf gpurun_out/abf/p
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/abf/p -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no_eval > gpurun_out/abf/$lib.prof.log 2>&1 || { tail -5 gpurun_out/abf/$lib.prof.log; exit 2; }
  f=$(find gpurun_out/abf/p -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/abf/$lib.kernel_stats.csv
  rm -rf gpurun_out/abf/p
  python3 - gpurun_out/abf/$lib.kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:6]:
    print(f'   {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:60]}')
PY
done
