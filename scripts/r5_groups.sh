#!/bin/bash
# pipelined rollout (--rollout_groups) A/B in the headline bench (phase timers on for the breakdown)
set -o pipefail
cd $GRAFT_REPO_ROOT
for g in 1 2 4 1 2; do
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no_eval --rollout_groups $g > gpurun_out/groups_$g.log 2>&1 || { tail -5 gpurun_out/groups_$g.log; exit 1; }
  python3 - $g <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/groups_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("groups", sys.argv[1], "value", d["value"], "ms", d["ms_per_step"], "phases", d.get("phase_ms_per_step"))
PY
done
