# PMC passes (one counter group per rocprofv3 run, kernel-trace only) over a command, summed
# per kernel name: bash tools/gpu_pmc_cmd.sh OUT FILTER "python cmd args" "PASS1" "PASS2" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$1; FILT=$2; CMD=$3; shift 3
rm -rf gpurun_out/$OUT; mkdir -p gpurun_out/$OUT
i=0
for PASS in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $PASS -d gpurun_out/$OUT/p$i -o run --output-format csv -- $CMD > gpurun_out/$OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/$OUT/p$i.log; exit 1; }
done
python3 - "$OUT" "$FILT" <<'PY'
import csv, glob, collections, sys
out, filt = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(set)
for f in glob.glob(f"gpurun_out/{out}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if filt not in k: continue
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k].add(r.get("Dispatch_Id", ""))
for k, d in vals.items():
    print(k, "dispatches", len(calls[k]))
    for c, v in sorted(d.items()): print("   %-24s %16.0f" % (c, v))
PY
