#!/bin/bash
# update-path fusion: PPO / Adam GPU tests, then the bench under rocprof
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_fuse.log 2>&1 || { tail -30 gpurun_out/pytest_fuse.log; exit 1; }
tail -2 gpurun_out/pytest_fuse.log
rm -rf gpurun_out/benchab
AB_LIBS="libmatdcml.so libmatdcml.so" bash scripts/r5_benchab.sh || exit 2
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/benchab/libmatdcml_w32.kernel_stats.csv")))
for r in rows:
    if any(k in r["Name"] for k in ("grad_reduce", "adam", "pack_weights", "Fill")):
        print(f'{float(r["TotalDurationNs"])/4/1e6:7.3f} ms/iter {int(r["Calls"])//4:4d} calls  {r["Name"][:60]}')
PY
