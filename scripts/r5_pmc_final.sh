#!/bin/bash
# round-5 final PMC: the four training kernels (tests/bench_train_kernels.py) and the speculative decode
# (scripts/decode_time.py at 256 x 33), one rocprofv3 --pmc pass per counter group (scripts/pmc.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc
bash scripts/pmc.sh > /dev/null || exit 1
mv gpurun_out/pmc/summary.txt gpurun_out/pmc_train_summary.txt
rm -rf gpurun_out/pmc
PMC_PROG="scripts/decode_time.py 33,2,2,256" bash scripts/pmc.sh > /dev/null || exit 2
mv gpurun_out/pmc/summary.txt gpurun_out/pmc_decode_summary.txt
cat gpurun_out/pmc_train_summary.txt gpurun_out/pmc_decode_summary.txt
