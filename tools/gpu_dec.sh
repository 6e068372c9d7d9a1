# decode A/B timing + PMC passes of the v8 decoder (run under gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/dec_ab.py > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
cat gpurun_out/ab.log
i=0
for PASS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
            "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $PASS -d gpurun_out/dpmc/p$i -o run --output-format csv -- python tools/dec_ab.py --variants 8x4 --rounds 1 --iters 2 > gpurun_out/dpmc_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/dpmc_p$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
vals = collections.defaultdict(list)
for f in glob.glob("gpurun_out/dpmc/p*/**/run_counter_collection.csv", recursive=True) + glob.glob("gpurun_out/dpmc/p*/run_counter_collection.csv"):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if "decode" not in k: continue
        per[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, d, c), v in per.items(): vals[(k, c)].append(v)
for (k, c), v in sorted(vals.items()):
    print("%-16s %-22s %16.0f" % (k, c, sum(v) / len(v)))
PY
