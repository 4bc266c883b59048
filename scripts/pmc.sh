set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc/list.txt 2>&1 || true
grep -oE "(SQ|TCC|TCP|GRBM)_[A-Z0-9_]+" $R/gpurun_out/pmc/list.txt | sort -u > $R/gpurun_out/pmc/names.txt || true
LIBS=${PMC_LIBS:-libmatdcml.so}
for lib in $LIBS; do
i=0
PROG=${PMC_PROG:-tests/bench_train_kernels.py}
SETS=${PMC_SETS:-"SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS,SQ_INSTS_SALU,SQ_INSTS_VMEM,SQ_BUSY_CYCLES TCC_EA0_ATOMIC_sum,TCC_HIT_sum,TCC_MISS_sum"}
for set in $SETS; do
  set=${set//,/ }
  i=$((i+1))
  MAT_DCML_LIBNAME=$lib timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc/$lib/p$i -o run -- python3 $R/$PROG > $R/gpurun_out/pmc/$lib.p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
done
cd $R
python3 - <<'PY'
import csv, glob, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for f in glob.glob("gpurun_out/pmc/*/p*/**/*counter_collection.csv", recursive=True):
    lib = f.split("/")[2]
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", r.get("Kernel-Name", ""))
        mk = re.search(r"mat_\w+(<[^>]*>)?", k)
        if not mk: continue
        k = lib + " " + mk.group(0)
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
with open("gpurun_out/pmc/summary.txt", "w") as out:
    for k, d in agg.items():
        out.write(k + "\n")
        for c, v in sorted(d.items()):
            out.write(f"   {c:28s} {v / max(cnt[k][c],1):16.1f}  (per dispatch)\n")
print(open("gpurun_out/pmc/summary.txt").read())
PY
find gpurun_out/pmc -name "*.csv" -size +5M -delete
