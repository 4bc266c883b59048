#!/bin/bash
# usage: scripts/gpu_call.sh OUTFILE TIMEOUT 'command'
# Runs one gpurun call; retries only while no box / slot is free (gpurun's own exit 3 with no verdict from the
# command) or on a transient harness failure — never when the command itself ran and failed.
out=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1
  rc=$?
  if grep -q "status=fail\|status=ok\|status=timeout\|status=refused" $out; then echo "rc=$rc" >> $out; exit $rc; fi
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $out; then echo "rc=$rc" >> $out; exit $rc; fi
  sleep 150
done
