#!/bin/bash
# Round-4 close-out: the round-end rehearsal (GPU tests, smoke, default bench, kernel stats), then every config.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/final_check.sh || exit $?
bash scripts/configs_bench.sh | cut -c1-300 || exit 9
