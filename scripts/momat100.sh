#!/bin/bash
# Multi-objective MAT at the reference's native DCML config (100 workers) vs the published MOMAT curves
# (data/dcml_benchmark/momat_{ct,payment}.csv, 800 k env steps).  Runs, each under its own time limit:
#   momat / dmomat with the reference argv (8 envs, T 50, 15 epochs x 4 minibatches, lr 5e-5): 1 M env steps =
#   2500 PPO updates, the reference's own sample budget;  then momat at 256 envs for a long run.
# MOMAT_RUNS overrides the list ("name:algo:envs:steps:extra-args" entries).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/momat100
mkdir -p $O
RUNS=${MOMAT_RUNS:-"momat8:momat:8:1000000: dmomat8:dmomat:8:1000000:"}
for r in $RUNS; do
  IFS=: read name algo envs steps extra <<< "$r"
  timeout -k 10 ${MOMAT_TIMEOUT:-420} python -u DCML_MAT_Train.py --algorithm_name $algo --n_workers 100 \
    --n_rollout_threads $envs --num_env_steps $steps --log_interval 5 --save_interval 100000 \
    --results_dir $O/$name ${extra//,/ } > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  grep -E "FPS" $O/$name.log | tail -n 1
  f=$(find $O/$name -name summary.json | head -1)
  cp "$f" $O/summary_$name.json
  find $O/$name -name "*.pt" -delete
done
python3 scripts/momat_compare.py $O/summary_*.json | tee $O/compare.md
