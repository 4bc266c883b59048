set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 400 python -m pytest tests/test_gpu_ppo.py -x -q > gpurun_out/t_ppo.log 2>&1; rc=$?; tail -25 gpurun_out/t_ppo.log; [ $rc = 0 ] || exit 2
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -3 gpurun_out/bench.log; [ $rc = 0 ] || exit 4
timeout -k 10 300 python train_smac.py --num_env_steps 6400 --n_rollout_threads 32 --episode_length 100 --ppo_epoch 2 --log_interval 1 --profile_phases --results_dir /tmp/smac > gpurun_out/smac.log 2>&1; rc=$?; tail -12 gpurun_out/smac.log; exit $rc
