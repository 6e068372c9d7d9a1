# LDS utilisation counters for the decode kernel (run under gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
i=0
for PASS in "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_INST_CYCLES_VMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $PASS -d gpurun_out/lpmc/p$i -o run --output-format csv -- python tools/dec_ab.py --variants ${1:-16x2} --rounds 1 --iters 2 > gpurun_out/lpmc_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/lpmc_p$i.log; }
done
python - <<'PY'
import csv, glob, collections
vals = collections.defaultdict(list)
for f in glob.glob("gpurun_out/lpmc/p*/run_counter_collection.csv"):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if "decode" not in k: continue
        per[(k[:24], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, d, c), v in per.items(): vals[(k, c)].append(v)
for (k, c), v in sorted(vals.items()):
    print("%-24s %-22s %16.0f" % (k, c, sum(v) / len(v)))
PY
