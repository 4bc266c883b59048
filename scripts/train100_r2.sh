set -o pipefail
# Round-2 100-worker run (the reference's native DCML config) on the fused HIP trainer: 4x the round-1 budget
# (30.7 M env steps), then the reference benchmark sweep for the trained policy and the fixed heuristic.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2_train100
mkdir -p $O
timeout -k 10 960 python -u DCML_MAT_Train.py --n_workers 100 --n_rollout_threads 256 --num_env_steps 30720000 \
  --lr 5e-4 --critic_lr 5e-4 --save_interval 400 --log_interval 10 --results_dir $O > $O/train.log 2>&1 || { tail -20 $O/train.log; exit 1; }
grep -E "FPS|average rewards" $O/train.log | tail -n 4
CK=$(ls -t $O/DCML/AS/mat/check/run1/models/transformer_*.pt | head -n 1)
echo "checkpoint $CK"
cp $O/DCML/AS/mat/check/run1/logs/summary.json $O/summary_mat.json
timeout -k 10 200 python DCML_MAT_ALT_Benchmark.py --model_dir $CK --out $O/mat_AW.npy --json $O/mat_AW.json > $O/bench_mat.log 2>&1 || { tail $O/bench_mat.log; exit 2; }
timeout -k 10 200 python DCML_MAT_ALT_Benchmark.py --policy fixed --out $O/fixed_AW.npy --json $O/fixed_AW.json > $O/bench_fixed.log 2>&1 || { tail $O/bench_fixed.log; exit 3; }
grep -E "ct:|latency" $O/bench_mat.log | tail -4; grep "ct:" $O/bench_fixed.log | tail -2
cp $CK $O/
find $O -name "*.pt" -path "*run1*" -delete
