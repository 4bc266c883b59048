set -o pipefail
# Native reduction unit test, the whole GPU test suite, kernel micro-benches, 1-GPU bench with phases.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
(cd tests/native && hipcc -O3 --offload-arch=gfx950 -Wno-unused-result dpp_reduce_test.hip -o /tmp/dpp_t) && timeout -k 5 60 /tmp/dpp_t || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 2; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python tests/bench_train_kernels.py || exit 3
timeout -k 10 200 python tests/bench_decode.py 2>&1 | grep "cap=1:" || exit 4
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --phases > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 5; }
tail -2 gpurun_out/bench.log | cut -c1-400
