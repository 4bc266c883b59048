set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MAT_DCML_GRAD_COPIES=0 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no_eval > gpurun_out/b0.log 2>&1; echo "copies0 rc=$?"; tail -n 1 gpurun_out/b0.log
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no_eval > gpurun_out/b8.log 2>&1; echo "copies8 rc=$?"; grep -v amdgpu.ids gpurun_out/b8.log | tail -n 12
exit 0
