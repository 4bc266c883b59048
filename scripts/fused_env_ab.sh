# GPU check of the fused planar-surrogate step: parity tests, then HalfCheetah 6x1 runner FPS fused vs torch+hipGraph.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fused_env
timeout -k 10 300 python -u -m pytest tests/test_mujoco.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/fused_env/pytest.txt 2>&1 || { tail -n 40 gpurun_out/fused_env/pytest.txt; exit 1; }
tail -n 3 gpurun_out/fused_env/pytest.txt
for f in 1 0; do
  MAT_DCML_ENV_FUSED=$f timeout -k 10 200 python -u train_mujoco.py --scenario HalfCheetah-v2 --agent_conf 6x1 \
    --n_rollout_threads 128 --episode_length 100 --num_env_steps 64000 --num_mini_batch 4 --ppo_epoch 5 \
    --log_interval 1 --eval_interval 1000 --episode_limit 200 --results_dir gpurun_out/fused_env/results_$f \
    > gpurun_out/fused_env/train_fused$f.log 2>&1 || exit $?
  echo "fused=$f"; grep FPS gpurun_out/fused_env/train_fused$f.log | tail -n 2
done
