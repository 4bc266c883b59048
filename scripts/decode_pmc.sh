#!/bin/bash
# PMC counters of the rollout decode kernel (tests/bench_decode.py at L=33): SQ wait / instruction mix, then the
# instruction-cache counters if this rocprofv3 lists them.  One rocprofv3 pass per counter group.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc/list.txt 2>&1 || true
grep -oE "(SQ|SQC|TCC|TCP|GRBM)_[A-Z0-9_]+" $R/gpurun_out/pmc/list.txt | sort -u > $R/gpurun_out/pmc/names.txt || true
SETS="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_BUSY_CYCLES SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_WAIT_INST_LDS"
if grep -qx SQC_ICACHE_MISSES $R/gpurun_out/pmc/names.txt && grep -qx SQC_ICACHE_HITS $R/gpurun_out/pmc/names.txt; then
  SETS="$SETS SQC_ICACHE_MISSES,SQC_ICACHE_HITS"
fi
if grep -qx SQ_IFETCH $R/gpurun_out/pmc/names.txt; then SETS="$SETS SQ_IFETCH,SQ_WAVES"; fi
i=0
for set in $SETS; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc ${set//,/ } --output-format csv -d $R/gpurun_out/pmc/dec/p$i -o run -- python3 $R/tests/bench_decode.py 33 > $R/gpurun_out/pmc/dec.p$i.log 2>&1 || { echo "pass $i ($set) failed rc=$?"; exit 1; }
done
cd $R
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(float); cnt = collections.defaultdict(int)
for f in glob.glob("gpurun_out/pmc/dec/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mat_decode_kernel" not in r.get("Kernel_Name", ""): continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
with open("gpurun_out/pmc/decode_summary.txt", "w") as out:
    for c, v in sorted(agg.items()):
        out.write(f"   {c:28s} {v / max(cnt[c], 1):16.1f}  (per dispatch)\n")
print(open("gpurun_out/pmc/decode_summary.txt").read())
PY
find gpurun_out/pmc -name "*.csv" -size +5M -delete
