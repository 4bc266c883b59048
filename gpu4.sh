set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats.csv
find gpurun_out/prof -name "*kernel_trace.csv" -exec rm {} \;
head -40 gpurun_out/kernel_stats.csv | cut -c1-220
exit $rc
