#!/bin/bash
# 32-worker MAT-AS training runs, then every saved checkpoint on the benchmark protocol against
# the fixed heuristic on Sample_1 AND the held-out Sample_2..10 (+ the heuristic frontier), selected on held-out.
# TRAIN_CFGS: space-separated "name:steps:extra,args".
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5_train32
mkdir -p $O
export TMPDIR=/tmp
for cfg in ${TRAIN_CFGS:-"b3d:51200000:--lr,5e-4,--critic_lr,5e-4,--use_linear_lr_decay,--reward_beta,3"}; do
  IFS=: read name steps extra <<< "$cfg"
  timeout -k 10 ${TRAIN_TIMEOUT:-540} python -u DCML_MAT_Train.py --n_workers 32 --n_rollout_threads 256 \
    --num_env_steps $steps --save_interval 500 --log_interval 100 --results_dir $O/$name ${extra//,/ } \
    > $O/train_$name.log 2>&1 || { tail -20 $O/train_$name.log; exit 1; }
  grep -E "FPS" $O/train_$name.log | tail -n 1
done
[ -n "$NO_EVAL" ] && exit 0
cks=$(find $O -name "transformer_*.pt" | grep -v "transformer_0.pt" | sort -V)
timeout -k 10 900 python -u scripts/eval_ckpts.py --n_workers 32 --json $O/eval_ckpts.json $cks > $O/eval_ckpts.md 2>&1 || { tail $O/eval_ckpts.md; exit 2; }
tail -4 $O/eval_ckpts.md
