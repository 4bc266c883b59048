#!/bin/bash
# final unprofiled bench numbers: headline (10 timed steps), 100 / 128 workers, SMAC
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/configs_final
timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --no_eval > gpurun_out/configs_final/w32.log 2>&1 || { tail -5 gpurun_out/configs_final/w32.log; exit 1; }
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --no_eval --n_workers 100 > gpurun_out/configs_final/w100.log 2>&1 || { tail -5 gpurun_out/configs_final/w100.log; exit 2; }
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --no_eval --n_workers 128 > gpurun_out/configs_final/w128.log 2>&1 || { tail -5 gpurun_out/configs_final/w128.log; exit 3; }
timeout -k 10 400 python3 bench.py --config smac --steps 3 --warmup 1 --no_eval > gpurun_out/configs_final/smac.log 2>&1 || { tail -5 gpurun_out/configs_final/smac.log; exit 4; }
for f in w32 w100 w128 smac; do
  python3 - gpurun_out/configs_final/$f.log $f <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"{sys.argv[2]:5s} {d['value']:10.0f} env-steps/s  {d['ms_per_step']:8.2f} ms/step  steps {d['steps']}")
PY
done
