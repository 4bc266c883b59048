#!/bin/bash
# Kernel stats of a 3-step headline bench (rocprofv3) + the CT phase profile (libmatdcml_ctprof.so, -DMDL_CT_PROF).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/kstats.sh || exit 1
bash scripts/ct_prof.sh || exit 2
