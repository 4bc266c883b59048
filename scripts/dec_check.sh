set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_decode.py -x -q -s > gpurun_out/t_dec.log 2>&1; rc=$?; grep -E "passed|failed|us|ms|Error" gpurun_out/t_dec.log | tail -n 12; [ $rc = 0 ] || exit 2
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -n 1 gpurun_out/bench.log; exit $rc
