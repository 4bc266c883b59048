set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 300 python -m pytest tests/test_gpu_decode.py -x -q -s > gpurun_out/pytest_decode.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_decode.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --phases > gpurun_out/bench_auto.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_auto.log
exit $rc
