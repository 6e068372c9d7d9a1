# Adaptive nybble encode writer: which kernel runs, and its counters (k_nyb_enc_wtile<true> vs k_fsm_write<0>)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r5z3}
for v in 0 1; do
  rm -rf gpurun_out/${T}_sq$v
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/${T}_sq$v -o run --output-format csv -- python tools/abl_time.py --stage nyb_adaptive --cfg C1 --nary 0 --iters 2 --warm 1 --opt nyb_wtile_off=$v > gpurun_out/${T}_sq$v.log 2>&1 || { tail -5 gpurun_out/${T}_sq$v.log; exit 1; }
  python - gpurun_out/${T}_sq$v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    print(sys.argv[1][-4:], k[:40], {c: round(v / n[(k, c)]) for c, v in d.items()})
PY
done
