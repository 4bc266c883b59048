#!/bin/bash
# Round-5 start: occupancy A/B of the training backward (8 / 12 / 16 waves per workgroup), fresh PMC on the four
# training kernels (3200 x 33), kernel stats of the 100 / 128-worker benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libmatdcml.so libmatdcml_ab_nw12.so libmatdcml_ab_nw16.so libmatdcml_ab_watom.so libmatdcml_ab_nw12watom.so; do
  for L in 33 101; do
    echo -n "$lib " >> gpurun_out/train_micro.txt
    MAT_DCML_LIBNAME=$lib timeout -k 10 200 python3 tests/bench_train_kernels.py 3200 $L 10 >> gpurun_out/train_micro.txt 2>&1 || { tail gpurun_out/train_micro.txt; exit 1; }
  done
done
cat gpurun_out/train_micro.txt
for lib in libmatdcml_ab_nw12.so libmatdcml_ab_nw16.so; do
  MAT_DCML_LIBNAME=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_train_$lib.log 2>&1; echo "$lib pytest rc=$?"; tail -2 gpurun_out/pytest_train_$lib.log
done
PMC_SETS="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_BUSY_CYCLES SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_INSTS_SALU,SQ_WAVES SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_SMEM TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_ATOMIC_sum" PMC_LIBS="libmatdcml.so libmatdcml_ab_nw12.so" bash scripts/pmc.sh > gpurun_out/pmc_run.log 2>&1 || { tail -30 gpurun_out/pmc_run.log; exit 2; }
bash scripts/kstats_w100.sh || exit 3
