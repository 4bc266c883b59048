#!/bin/bash
# MOMAT at the reference argv (100 workers, 8 envs, T 50, 15 epochs x 4 minibatches, lr 5e-5, 1 M env steps) over
# 3 seeds, plus 3 seeds with --use_linear_lr_decay (mat_src/mat/config.py:278).  8 envs x 101 agents is a
# latency-bound shape that leaves the GPU mostly idle, so the six runs share the one GPU as six processes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/momat_seeds
mkdir -p $O
export TMPDIR=/tmp
pids=()
for cfg in "s1:--seed,1" "s2:--seed,2" "s3:--seed,3" "d1:--seed,1,--use_linear_lr_decay" "d2:--seed,2,--use_linear_lr_decay" "d3:--seed,3,--use_linear_lr_decay"; do
  name=${cfg%%:*}; extra=${cfg#*:}
  timeout -k 10 ${MOMAT_TIMEOUT:-1050} python -u DCML_MAT_Train.py --algorithm_name momat --n_workers 100 \
    --n_rollout_threads 8 --num_env_steps 1000000 --log_interval 5 --save_interval 100000 \
    --results_dir $O/$name ${extra//,/ } > $O/$name.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
for name in s1 s2 s3 d1 d2 d3; do
  grep -E "FPS" $O/$name.log | tail -n 1
  f=$(find $O/$name -name scalars.jsonl | head -1)
  [ -n "$f" ] && cp "$f" $O/scalars_$name.jsonl
done
find $O -name "*.pt" -delete
python3 scripts/momat_seeds.py momat=$O/scalars_s1.jsonl,$O/scalars_s2.jsonl,$O/scalars_s3.jsonl \
  momat_lrdecay=$O/scalars_d1.jsonl,$O/scalars_d2.jsonl,$O/scalars_d3.jsonl | tee $O/seeds.md
exit $rc
