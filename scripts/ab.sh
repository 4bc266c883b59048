set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for pers in 0 1; do
  echo "persistent=$pers"; MAT_DCML_PERSISTENT=$pers timeout -k 10 120 python tests/bench_train_kernels.py || exit 1
  MAT_DCML_PERSISTENT=$pers timeout -k 10 300 python bench.py --no_eval > gpurun_out/ab_$pers.log 2>&1 || exit 2
  python -c "import json;d=json.loads(open('gpurun_out/ab_$pers.log').read().strip().splitlines()[-1]);print('bench', d['value'], d['ms_per_step'])"
done
MAT_DCML_GRAD_COPIES=0 timeout -k 10 300 python bench.py --no_eval > gpurun_out/ab_c0.log 2>&1 || exit 3
python -c "import json;d=json.loads(open('gpurun_out/ab_c0.log').read().strip().splitlines()[-1]);print('copies0 bench', d['value'], d['ms_per_step'])"
