# Kernel-time profile of the MA-MuJoCo (Continuous action type) training loop: the rollout decode is fused,
# the teacher-forced update still runs in PyTorch eager — this shows how the iteration splits between them.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_mujoco
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_mujoco -o run -- \
  python3 -u $GRAFT_REPO_ROOT/train_mujoco.py --scenario HalfCheetah-v2 --agent_conf 6x1 --n_rollout_threads 128 \
  --episode_length 100 --num_env_steps 38400 --num_mini_batch 4 --ppo_epoch 5 --log_interval 1 --eval_interval 1000 \
  --episode_limit 200 --results_dir $GRAFT_REPO_ROOT/gpurun_out/prof_mujoco/results \
  > $GRAFT_REPO_ROOT/gpurun_out/prof_mujoco/train.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
grep -v amdgpu.ids gpurun_out/prof_mujoco/train.log | tail -n 4
mkdir -p gpurun_out/prof_mujoco_keep
find gpurun_out/prof_mujoco -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_mujoco_keep/ \;
cp gpurun_out/prof_mujoco/train.log gpurun_out/prof_mujoco_keep/
rm -rf gpurun_out/prof_mujoco
exit $rc
