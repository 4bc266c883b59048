#!/bin/bash
# chunk-order stagger A/B in the bench (rocprof kernel stats), then the long-seq / SMAC benches with the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/benchab
AB_LIBS="libmatdcml.so libmatdcml_ab_fwd0.so libmatdcml_ab_st2.so libmatdcml.so libmatdcml_ab_fwd0.so libmatdcml_ab_st2.so" bash scripts/r5_benchab.sh || exit 1
AB_LIBS="libmatdcml.so" TAG=w100 BENCH_ARGS="--n_workers 100" bash scripts/r5_benchab.sh || exit 2
d=gpurun_out/benchab/smac
timeout -k 10 400 python3 bench.py --config smac --steps 3 --warmup 1 --no_eval > $d.log 2>&1 || { tail -5 $d.log; exit 4; }
grep '"metric"' $d.log | cut -c1-220
cat gpurun_out/benchab/summary.txt
