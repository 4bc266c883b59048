set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest $1 -x -q -s > gpurun_out/one.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/one.log | tail -n 15; exit $rc
