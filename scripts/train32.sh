set -o pipefail
# 32-worker DCML (the headline config): train MAT-AS on one GPU, then the reference benchmark sweep (available
# workers) for the trained policy and the fixed heuristic; then a short multi-objective (momat) run for curves.
cd $GRAFT_REPO_ROOT
O=gpurun_out/train32
mkdir -p $O
timeout -k 10 420 python -u DCML_MAT_Train.py --n_workers 32 --n_rollout_threads 256 --num_env_steps 10240000 \
  --lr 5e-4 --critic_lr 5e-4 --save_interval 100 --log_interval 20 --results_dir $O > $O/train.log 2>&1 || { tail -20 $O/train.log; exit 1; }
grep -E "FPS|average rewards" $O/train.log | tail -n 4
CK=$(ls -t $O/DCML/AS/mat/check/run1/models/transformer_*.pt | head -n 1)
echo "checkpoint $CK"
cp $O/DCML/AS/mat/check/run1/logs/summary.json $O/summary_mat.json
timeout -k 10 200 python DCML_MAT_ALT_Benchmark.py --n_workers 32 --model_dir $CK --out $O/mat_AW.npy --json $O/mat_AW.json > $O/bench_mat.log 2>&1 || { tail $O/bench_mat.log; exit 2; }
timeout -k 10 200 python DCML_MAT_ALT_Benchmark.py --n_workers 32 --policy fixed --out $O/fixed_AW.npy --json $O/fixed_AW.json > $O/bench_fixed.log 2>&1 || { tail $O/bench_fixed.log; exit 3; }
grep -E "ct:|latency" $O/bench_mat.log | tail -4; grep "ct:" $O/bench_fixed.log | tail -2
cp $CK $O/
timeout -k 10 300 python -u DCML_MAT_Train.py --n_workers 32 --n_rollout_threads 256 --num_env_steps 5120000 \
  --algorithm_name momat --lr 5e-4 --critic_lr 5e-4 --save_interval 1000 --log_interval 5 --results_dir $O/mo > $O/train_momat.log 2>&1 || { tail -20 $O/train_momat.log; exit 4; }
cp $O/mo/DCML/AS/momat/check/run1/logs/summary.json $O/summary_momat.json
find $O -name "*.pt" -path "*run1*" -delete
tail -3 $O/train_momat.log
