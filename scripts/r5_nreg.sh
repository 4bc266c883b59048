#!/bin/bash
# main-wave register-resident matrices of the speculative decode (MAT_DCML_SPEC_NREG = the smallest tried)
set -o pipefail
cd $GRAFT_REPO_ROOT
for n in 0 2 4 6 8 4; do
  echo "== nreg >= $n"
  MAT_DCML_LIBNAME=libmatdcml_ab_nreg.so MAT_DCML_SPEC_NREG=$n timeout -k 10 120 python scripts/decode_time.py 2>&1 | grep decode || exit 1
done
