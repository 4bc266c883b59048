set -o pipefail
# One GPU call: gpu tests, 1-GPU bench (+ phase breakdown), rocprofv3 kernel stats. Extensions are built on the CPU host.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --phases > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -25 gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no_eval > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats.csv
find gpurun_out/prof -name "*kernel_trace.csv" -delete
head -25 gpurun_out/kernel_stats.csv | cut -d, -f1-8 | cut -c1-180
