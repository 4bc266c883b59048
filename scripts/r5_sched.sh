#!/bin/bash
# AMDGPU scheduler-strategy A/B: the speculative decode (decode_time.py) and the training kernels (in-bench rocprof)
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in libmatdcml.so libmatdcml_ab_decw_ilp.so libmatdcml_ab_decw_mmc.so libmatdcml_ab_decw_trk.so; do
  echo "== $lib"
  MAT_DCML_LIBNAME=$lib timeout -k 10 120 python scripts/decode_time.py 2>&1 | grep "decode\]" || exit 1
done
rm -rf gpurun_out/benchab
AB_LIBS="libmatdcml.so libmatdcml_ab_bwd_ilp.so libmatdcml_ab_bwd_mmc.so libmatdcml_ab_fwd_ilp.so" bash scripts/r5_benchab.sh || exit 2
