#!/bin/bash
# PMC counters of the rollout decode (tests/bench_decode.py at L=33) for the one-wave and the 4-wave kernel:
# instruction mix and wait cycles, one rocprofv3 pass per counter group.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp
SETS="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_WAIT_INST_LDS,SQ_WAVES,SQ_LDS_BANK_CONFLICT"
for arm in 1 0; do
  i=0
  for set in $SETS; do
    i=$((i+1))
    MAT_DCML_DECODE_WAVE=$arm timeout -s KILL 90 rocprofv3 --pmc ${set//,/ } --output-format csv -d $R/gpurun_out/pmc2/w$arm/p$i -o run -- python3 $R/tests/bench_decode.py 33 > $R/gpurun_out/pmc2/w$arm.p$i.log 2>&1 || { echo "pass $arm/$i ($set) failed rc=$?"; tail -5 $R/gpurun_out/pmc2/w$arm.p$i.log; exit 1; }
  done
done
cd $R
python3 - <<'PY'
import csv, glob, collections
for arm in ("1", "0"):
    agg = collections.defaultdict(float); cnt = collections.defaultdict(int)
    for f in glob.glob(f"gpurun_out/pmc2/w{arm}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "mat_decode" not in r.get("Kernel_Name", ""): continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
    w = agg.get("SQ_WAVES", 1) / max(cnt.get("SQ_WAVES", 1), 1)
    print("one-wave" if arm == "1" else "4-wave", "per dispatch, per wave:")
    for c, v in sorted(agg.items()):
        d = v / max(cnt[c], 1)
        print(f"   {c:24s} {d:16.1f}  per wave {d / w:12.1f}")
PY
find gpurun_out/pmc2 -name "*.csv" -size +5M -delete
