# wave-per-tile nybble writers: plain vs nt input loads (tree vs tools/_old), time and FETCH_SIZE
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r5g}
bash tools/gpu_ab_old.sh ${T} "nyb_static_step C1 0" || exit 1
for L in new old; do
  LIB=""; [ $L = old ] && LIB=tools/_old/libdc_core.so
  D=gpurun_out/${T}_fetch_$L; rm -rf $D
  DC_CORE_LIB=$LIB timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $D -o run --output-format csv -- python tools/abl_time.py --stage nyb_static_step --cfg C1 --nary 0 --iters 2 --warm 1 > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
  python - $D <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:30]
    if "nyb" not in k: continue
    agg[k] += float(r["Counter_Value"]); n[k] += 1
for k in agg: print(sys.argv[1][-10:], k, "FETCH_SIZE KiB per dispatch (raw)", round(agg[k] / n[k]))
PY
done
