set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats.csv
find gpurun_out/prof -name "*kernel_trace.csv" -exec rm {} \;
head -30 gpurun_out/kernel_stats.csv | cut -d, -f1-8 | cut -c1-200
[ $rc = 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; exit $rc
