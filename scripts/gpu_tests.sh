set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "mean step reward|passed|failed|Error" gpurun_out/pytest_gpu.log | tail -n 8; exit $rc
