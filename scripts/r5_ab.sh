#!/bin/bash
# A/B of library variants on the four training kernels: rocprofv3 kernel time (no host gaps) of
# tests/bench_train_kernels.py per library, at L = 33 (and L_LIST), then (optionally) the GPU training tests per variant.
#   AB_LIBS="libmatdcml.so libmatdcml_ab_x.so" L_LIST="33 101" AB_TESTS=1 bash scripts/r5_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for lib in ${AB_LIBS:-libmatdcml.so}; do
  for L in ${L_LIST:-33}; do
    d=gpurun_out/ab/${lib%.so}_L$L
    rm -rf $d
    MAT_DCML_LIBNAME=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 tests/bench_train_kernels.py 3200 $L 10 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    python3 - "$f" "$lib" "$L" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
want = {"mat_enc_fwd_ct<2, true>": "enc_fwd", "mat_dec_fwd_ct<2, true": "dec_fwd", "mat_dec_bwd_ct": "dec_bwd", "mat_enc_bwd_ct": "enc_bwd"}
out = {}
for r in rows:
    for k, v in want.items():
        if k in r["Name"]:
            out[v] = float(r["AverageNs"]) / 1e3
s = sum(out.values())
print(f"{sys.argv[2]:32s} L={sys.argv[3]:4s} " + " ".join(f"{k} {out.get(k, 0):7.1f}" for k in ("enc_fwd", "dec_fwd", "dec_bwd", "enc_bwd")) + f"  sum {s:7.1f} us")
PY
    find $d -name "*kernel_trace.csv" -delete
  done
done | tee gpurun_out/ab/summary.txt
if [ -n "$AB_TESTS" ]; then
  for lib in ${AB_LIBS}; do
    MAT_DCML_LIBNAME=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/pytest_$lib.log 2>&1; echo "$lib pytest rc=$?"; tail -1 gpurun_out/ab/pytest_$lib.log
  done
fi
