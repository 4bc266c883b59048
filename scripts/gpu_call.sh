#!/bin/bash
# usage: scripts/gpu_call.sh OUTFILE TIMEOUT 'command'
# Runs one gpurun call; retries only while no box / slot is free (gpurun's own exit 3 with no verdict from the
# command) or on a transient harness failure — never when the command itself ran and failed.  Every attempt first
# waits until the in-tree HIP library matches the sources (a snapshot taken mid-edit would ship a stale library).
out=$1; to=$2; cmd=$3
fresh() {
  python3 -c "import sys; sys.path.insert(0, '$(dirname "$0")/..'); from mat_dcml_amd.ops import kernels as k; \
sys.exit(0 if k._sidecar_stale(k._build_mod()) is None else 1)" 2>/dev/null
}
for i in $(seq 1 40); do
  for j in $(seq 1 40); do fresh && break; sleep 15; done
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1
  rc=$?
  if grep -q "status=fail\|status=ok\|status=timeout\|status=refused" $out; then echo "rc=$rc" >> $out; exit $rc; fi
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $out; then echo "rc=$rc" >> $out; exit $rc; fi
  sleep 120
done
