#!/bin/bash
# Multi-objective MAT at the reference's native DCML config (100 workers) vs the published MOMAT curves
# (data/dcml_benchmark/momat_{ct,payment}.csv, 800 k env steps).  ONE run per call (gpurun time limits):
#   MOMAT_RUN="name:algo:envs:steps:extra-args"  (extra args comma-separated), default the reference argv
#   (8 envs, T 50, 15 epochs x 4 minibatches, lr 5e-5) for 1 M env steps = 2500 PPO updates.
# logs/scalars.jsonl is written as the run goes, so the comparison also covers a run cut at its limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/momat100
mkdir -p $O
IFS=: read name algo envs steps extra <<< "${MOMAT_RUN:-momat8:momat:8:1000000:}"
timeout -k 10 ${MOMAT_TIMEOUT:-1000} python -u DCML_MAT_Train.py --algorithm_name $algo --n_workers 100 \
  --n_rollout_threads $envs --num_env_steps $steps --log_interval ${MOMAT_LOG:-5} --save_interval 100000 \
  --results_dir $O/$name ${extra//,/ } > $O/$name.log 2>&1
rc=$?
grep -E "FPS" $O/$name.log | tail -n 1
f=$(find $O/$name -name scalars.jsonl | head -1)
cp "$f" $O/scalars_$name.jsonl
find $O/$name -name "*.pt" -delete
python3 scripts/momat_compare.py $O/scalars_$name.jsonl | tee $O/compare_$name.md
exit $rc
