# Static nybble encode writer, a wave per tile (k_nyb_enc_wtile) vs a workgroup per tile
# (k_fsm_write, DC_OPT_NYB_WTILE_OFF=1): nybble parity tests, same-process A/B, SQ counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r5y}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "nybble" > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_ab.log
for r in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 150 python tools/abl_time.py --stage nyb_static_step --cfg C1 --nary 0 --iters 10 --warm 10 --opt nyb_wtile_off=$v --tag wtile_off=$v >> gpurun_out/${T}_ab.log 2>&1 || { tail -3 gpurun_out/${T}_ab.log; exit 1; }
  done
done
grep '^{' gpurun_out/${T}_ab.log | cut -c1-400
for v in 0 1; do
  rm -rf gpurun_out/${T}_sq$v
  DC_NYB_WTILE_OFF=$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/${T}_sq$v -o run --output-format csv -- python tools/abl_time.py --stage nyb_static_step --cfg C1 --nary 0 --iters 2 --warm 1 --opt nyb_wtile_off=$v > gpurun_out/${T}_sq$v.log 2>&1 || { tail -5 gpurun_out/${T}_sq$v.log; exit 1; }
  python - gpurun_out/${T}_sq$v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "write" not in k and "wtile" not in k and "nyb_tiles" not in k: continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    print(sys.argv[1], k[:40], {c: round(v / n[(k, c)]) for c, v in d.items()})
PY
done
