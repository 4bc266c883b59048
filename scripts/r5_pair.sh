#!/bin/bash
# PAIR layout of the speculative decode (act_dim <= 2): decode parity tests + latency, then the phase profile
set -o pipefail
cd $GRAFT_REPO_ROOT
rm -f gpurun_out/perf_guards.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pair.log 2>&1
rc=$?
grep -E "\[perf\]|passed|failed|Error|assert" gpurun_out/pytest_pair.log | head -30
[ $rc -eq 0 ] || exit $rc
MAT_DCML_LIBNAME=libmatdcml_ab_spprof.so timeout -k 10 120 python scripts/spec_prof.py 33,2,2,256 || exit 2
