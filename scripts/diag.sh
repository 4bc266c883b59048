set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest "tests/test_gpu_train.py::test_full_mat_fused_grads[5-77]" -q -s > gpurun_out/mfma.log 2>&1
MAT_DCML_LIBNAME=libvalu.so timeout -k 10 300 python -m pytest "tests/test_gpu_train.py::test_full_mat_fused_grads[5-77]" -q -s > gpurun_out/valu.log 2>&1
tail -n 3 gpurun_out/mfma.log; tail -n 3 gpurun_out/valu.log
exit 0
