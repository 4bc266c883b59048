#!/bin/bash
# MA-MuJoCo faulty-node training: agent 0 (bfoot) disabled during training, evaluated with and without the fault
set -o pipefail
mkdir -p gpurun_out/learn
timeout -k 10 330 python -u train_mujoco.py --scenario HalfCheetah-v2 --agent_conf 6x1 --agent_obsk 0 --n_rollout_threads 128 --episode_length 100 --num_env_steps 1200000 --num_mini_batch 4 --ppo_epoch 5 --lr 5e-4 --log_interval 5 --eval_interval 20 --faulty_node 0 --eval_faulty_node -1 0 --n_eval_rollout_threads 8 --eval_episodes 8 --episode_limit 200 --experiment_name faulty0 --results_dir gpurun_out/learn/results > gpurun_out/learn/mujoco_faulty0.log 2>&1
rc=$?; [ $rc = 0 ] || [ $rc = 124 ] || exit $rc
exit 0
