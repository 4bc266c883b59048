#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/ct_ab.txt
bash scripts/smac_check.sh || exit 1
bash scripts/ct_ab.sh || exit 1
