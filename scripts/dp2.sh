set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MAT_DCML_DIST_BACKEND=gloo MAT_DCML_SHARE_DEVICES=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 2 --warmup 1 --no_eval > gpurun_out/dp2.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/dp2.log | tail -n 5; exit $rc
