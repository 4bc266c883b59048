set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 300 python -m pytest tests/test_gpu_train.py -x -q > gpurun_out/pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_train.log
exit $rc
