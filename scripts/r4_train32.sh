#!/bin/bash
# 32-worker MAT-AS training with the current fused trainer, then every saved checkpoint of each
# run on the benchmark protocol vs the fixed heuristic (scripts/eval_ckpts.py).  TRAIN_CFGS: space-separated
# "name:steps:extra,args" (default: lr 5e-4 constant, and lr 5e-4 with linear decay; 51.2 M env steps each).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4_train32
mkdir -p $O
export TMPDIR=/tmp
for cfg in ${TRAIN_CFGS:-"c5e4:51200000:--lr,5e-4,--critic_lr,5e-4" "d5e4:51200000:--lr,5e-4,--critic_lr,5e-4,--use_linear_lr_decay"}; do
  IFS=: read name steps extra <<< "$cfg"
  timeout -k 10 ${TRAIN_TIMEOUT:-540} python -u DCML_MAT_Train.py --n_workers 32 --n_rollout_threads 256 \
    --num_env_steps $steps --save_interval 500 --log_interval 50 --results_dir $O/$name ${extra//,/ } \
    > $O/train_$name.log 2>&1 || { tail -20 $O/train_$name.log; exit 1; }
  grep -E "FPS" $O/train_$name.log | tail -n 1
  cp $(find $O/$name -name summary.json | head -1) $O/summary_$name.json 2>/dev/null
done
[ -n "$NO_EVAL" ] && exit 0
cks=$(find $O -name "transformer_*.pt" | sort -V)
timeout -k 10 400 python -u scripts/eval_ckpts.py --n_workers 32 --json $O/eval_ckpts.json $cks | tee $O/eval_ckpts.md || exit 2
