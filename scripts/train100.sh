set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/train100
timeout -k 10 840 python DCML_MAT_Train.py --n_workers 100 --n_rollout_threads 256 --num_env_steps 7680000 \
  --lr 5e-4 --critic_lr 5e-4 --save_interval 50 --log_interval 25 --results_dir gpurun_out/train100 \
  > gpurun_out/train100/train.log 2>&1
echo "train rc=$?"
grep -E "FPS|average rewards" gpurun_out/train100/train.log | tail -n 6
CK=$(ls -t gpurun_out/train100/DCML/AS/mat/check/run1/models/transformer_*.pt | head -n 1)
echo "checkpoint $CK"
timeout -k 10 200 python DCML_MAT_ALT_Benchmark.py --model_dir $CK --out gpurun_out/train100/mat_AW.npy --json gpurun_out/train100/mat_AW.json > gpurun_out/train100/bench_mat.log 2>&1; echo "bench rc=$?"
timeout -k 10 200 python DCML_MAT_ALT_Benchmark.py --policy fixed --out gpurun_out/train100/fixed_AW.npy --json gpurun_out/train100/fixed_AW.json > gpurun_out/train100/bench_fixed.log 2>&1
grep -E "ct:|latency" gpurun_out/train100/bench_mat.log; grep "ct:" gpurun_out/train100/bench_fixed.log
find gpurun_out/train100 -name "transformer_*.pt" ! -name "$(basename $CK)" -delete
