#!/bin/bash
# Round-3 check: every GPU test, smoke(), default bench (with eval block), kernel stats, A/B of library variants.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/ct_ab.txt
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 2; }
tail -1 gpurun_out/smoke.log | cut -c1-200
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 3; }
tail -1 gpurun_out/bench.log | cut -c1-240
bash scripts/kstats.sh || exit 4
[ -n "$(ls mat_dcml_amd/_lib/libmatdcml_ab_*.so 2>/dev/null)" ] && { bash scripts/ct_ab.sh || exit 5; }
exit 0
