set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_train.py tests/test_gpu_ppo.py -x -q > gpurun_out/t_train.log 2>&1; rc=$?; tail -n 4 gpurun_out/t_train.log; [ $rc = 0 ] || exit 2
echo kern; timeout -k 10 120 python tests/bench_train_kernels.py || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -n 1 gpurun_out/bench.log; exit $rc
