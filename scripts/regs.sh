#!/bin/bash
# Register / scratch usage of the training kernels of one translation unit (hipcc -Rpass-analysis, CPU only).
# usage: scripts/regs.sh mat_dec_ct_bwd.hip 'mat_dec_bwd_ctILi2ELi1ELb0'
cd "$(dirname "$0")/../mat_dcml_amd/csrc"
extra=""
case "$1" in mat_dec_ct_bwd.hip|mat_enc_ct.hip) extra="-mllvm -amdgpu-use-amdgpu-trackers=1";; esac
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -munsafe-fp-atomics -Wno-unused-result \
  -fvisibility=hidden $extra $MAT_DCML_BWD_FLAGS -c "$1" -o /tmp/regs_$$.o -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep remark | sed 's/.*remark: *//; s/ \[-Rpass.*//' | awk -v pat="$2" '/Function Name/{show = index($0, pat) > 0} show'
rm -f /tmp/regs_$$.o
