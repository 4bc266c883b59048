#!/bin/bash
# captured decode-pack rebuild: GPU tests that step the optimizer between decodes, then the bench phases (graph on /
# off)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "runner or trainer or bench or smoke or rollout or mpe or smac or mujoco or determinism" > gpurun_out/pytest_packgraph.log 2>&1 || { tail -30 gpurun_out/pytest_packgraph.log; exit 1; }
tail -2 gpurun_out/pytest_packgraph.log
for g in 1 0 1; do
  MAT_DCML_PACK_GRAPH=$g timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no_eval > gpurun_out/pg_$g.log 2>&1 || { tail -5 gpurun_out/pg_$g.log; exit 2; }
  python3 - $g <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/pg_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("pack_graph", sys.argv[1], "value", d["value"], "ms", d["ms_per_step"], "phases", d.get("phase_ms_per_step"))
PY
done
