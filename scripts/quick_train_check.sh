set -o pipefail
# Training-kernel change check: numerics tests, kernel micro-bench, 1-GPU bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_ppo.py -x -q --timeout 120 --timeout-method thread > gpurun_out/qt_test.log 2>&1 || { tail -30 gpurun_out/qt_test.log; exit 1; }
tail -1 gpurun_out/qt_test.log
timeout -k 10 120 python tests/bench_train_kernels.py || exit 2
timeout -k 10 300 python bench.py --no_eval > gpurun_out/qt_bench.log 2>&1 || { tail -20 gpurun_out/qt_bench.log; exit 3; }
python -c "import json;d=json.loads(open('gpurun_out/qt_bench.log').read().strip().splitlines()[-1]);print('bench', d['value'], d['ms_per_step'])"
