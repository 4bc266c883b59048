#!/bin/bash
# GPU check of the MuJoCo / football envs + runners (short runs, each under its own time limit)
set -o pipefail
mkdir -p gpurun_out/envs
timeout -k 10 120 python -u -m pytest tests/test_mujoco.py tests/test_football.py -m gpu -x -v --timeout 100 --timeout-method thread -p no:cacheprovider > gpurun_out/envs/pytest.log 2>&1 || exit $?
timeout -k 10 240 python -u train_mujoco.py --scenario HalfCheetah-v2 --agent_conf 6x1 --n_rollout_threads 128 --episode_length 100 --num_env_steps 64000 --num_mini_batch 4 --ppo_epoch 5 --log_interval 1 --eval_interval 2 --eval_faulty_node -1 0 --n_eval_rollout_threads 5 --eval_episodes 5 --episode_limit 200 --results_dir gpurun_out/envs/results > gpurun_out/envs/mujoco.log 2>&1 || exit $?
timeout -k 10 240 python -u train_football.py --n_rollout_threads 128 --n_eval_rollout_threads 32 --episode_length 100 --num_env_steps 64000 --ppo_epoch 5 --log_interval 1 --eval_interval 2 --results_dir gpurun_out/envs/results > gpurun_out/envs/football.log 2>&1 || exit $?
