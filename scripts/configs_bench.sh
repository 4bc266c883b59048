set -o pipefail
# Every BASELINE config that fits one GPU: 32 / 100 / 128 workers DCML and the SMAC 27m_vs_30m stress env.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/configs
for w in 32 100 128; do
  timeout -k 10 300 python -u bench.py --n_workers $w --steps 3 --warmup 1 --no_eval > gpurun_out/configs/dcml_w$w.log 2>&1 || { tail -20 gpurun_out/configs/dcml_w$w.log; exit 1; }
  tail -1 gpurun_out/configs/dcml_w$w.log
done
timeout -k 10 300 python -u bench.py --config smac --steps 3 --warmup 1 --no_eval > gpurun_out/configs/smac.log 2>&1 || { tail -20 gpurun_out/configs/smac.log; exit 2; }
tail -1 gpurun_out/configs/smac.log
