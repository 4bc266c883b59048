set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 300 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --phases > gpurun_out/bench_auto.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_auto.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_torchpath -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
find gpurun_out/prof_torchpath -name "*stats*" | head
exit $rc
