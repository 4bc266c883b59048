#!/bin/bash
# Round-6 training run + held-out checkpoint selection.
#   W=100 STEPS=40960000 BETA=1 SAVE=400 LR=5e-4 TMAX=780 bash scripts/r6_train.sh
# Trains MAT-AS with the reference argv (DCML_MAT_Train.py) at W workers, 256 envs, linear LR decay, reward weights
# alpha 99 / beta BETA, then (EVAL_N > 0) evaluates the last EVAL_N checkpoints on the reference benchmark protocol (Sample_1 +
# held-out Sample_2..10 + the heuristic's frontier, scripts/eval_ckpts.py) and keeps the held-out pick.
set -o pipefail
cd $GRAFT_REPO_ROOT
W=${W:-100}; STEPS=${STEPS:-40960000}; BETA=${BETA:-1}; SAVE=${SAVE:-400}; LR=${LR:-5e-4}; TMAX=${TMAX:-780}
EVAL_N=${EVAL_N:-6}; SEED=${SEED:-1}
O=gpurun_out/r6_train${W}_b${BETA}_s${SEED}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 $TMAX python -u DCML_MAT_Train.py --n_workers $W --n_rollout_threads 256 --num_env_steps $STEPS \
  --lr $LR --critic_lr $LR --use_linear_lr_decay --reward_beta $BETA --seed $SEED --save_interval $SAVE \
  --log_interval 50 --results_dir $O > $O/train.log 2>&1 || { tail -20 $O/train.log; exit 1; }
grep -E "FPS" $O/train.log | tail -n 1 > $O/fps.txt
cat $O/fps.txt
if [ "$EVAL_N" = 0 ]; then exit 0; fi   # train only: evaluate in a later call (scripts/eval_ckpts.py)
CKS=$(ls -v $O/DCML/AS/mat/check/run1/models/transformer_*.pt | tail -n $EVAL_N)
timeout -k 10 ${EVAL_TMAX:-360} python -u scripts/eval_ckpts.py --n_workers $W --json $O/eval.json $CKS > $O/eval.md 2>&1 || { tail -20 $O/eval.md; exit 2; }
cat $O/eval.md
SEL=$(python -c "import json; print(json.load(open('$O/eval.json'))['selected_on_heldout'])")
cp $SEL $O/selected_$(basename $SEL)
find $O/DCML -name "trainer_state_*.pt" -delete
find $O/DCML -name "env_state_*" -delete
