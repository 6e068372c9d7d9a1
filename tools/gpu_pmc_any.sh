# PMC passes for the decode kernel with arbitrary counter groups: bash tools/gpu_pmc_any.sh VARIANT "PASS1" "PASS2" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
VAR=$1; shift
rm -rf gpurun_out/apmc
i=0
for PASS in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $PASS -d gpurun_out/apmc/p$i -o run --output-format csv -- python tools/dec_ab.py --variants $VAR --rounds 1 --iters 2 > gpurun_out/apmc_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/apmc_p$i.log; }
done
python - <<'PY'
import csv, glob, collections
vals = collections.defaultdict(list)
for f in glob.glob("gpurun_out/apmc/p*/run_counter_collection.csv"):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if "decode" not in k: continue
        per[(k[:24], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, d, c), v in per.items(): vals[(k, c)].append(v)
for (k, c), v in sorted(vals.items()):
    print("%-24s %-26s %16.0f" % (k, c, sum(v) / len(v)))
PY
