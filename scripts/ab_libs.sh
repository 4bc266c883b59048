set -o pipefail
# A/B of the training-kernel variants: numerics tests (default selection), kernel micro-bench and full bench each.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_test.log 2>&1 || { tail -30 gpurun_out/ab_test.log; exit 1; }
tail -1 gpurun_out/ab_test.log
for v in ${VARIANTS:-base o2}; do
  echo "=== $v"
  export MAT_DCML_TRAIN_VARIANT=$v
  timeout -k 10 120 python tests/bench_train_kernels.py || exit 2
  timeout -k 10 300 python bench.py --no_eval > gpurun_out/ab_bench_$v.log 2>&1 || { tail -20 gpurun_out/ab_bench_$v.log; exit 3; }
  python -c "import json;d=json.loads(open('gpurun_out/ab_bench_$v.log').read().strip().splitlines()[-1]);print('bench', d['value'], d['ms_per_step'])"
done
