# Round-6 profiling call (gpu_profile5.sh + C3's rocprof and PMC summaries) (run under gpurun): every GPU test and smoke(); for the C2 bench line,
# C4 and C5 (fused): rocprofv3 --kernel-trace --stats of the bench command and PMC passes
# (FETCH_SIZE, WRITE_SIZE, an SQ group; one rocprofv3 run each) summarised as the JSON bench.py
# cites (profiles/INDEX.json, updated here first so the lines after cite these); then the bench
# lines: C2 with its CPU baseline, C3-C5, the C5 two stages, nybble static and adaptive (with
# their own PMC traffic and rocprof stats). Everything it writes is also copied to
# gpurun_out/profiles_TAG/ (the box's profiles/ does not travel back).
# usage: bash tools/gpu_profile5.sh TAG [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r6z}
OUT=gpurun_out/profiles_${TAG}
mkdir -p gpurun_out $OUT profiles
GiB=1073741824
if [ -z "$2" ]; then
  bash tools/gpu_verify.sh ${TAG} || exit 1
fi
index_add() {   # prepend files to profiles/INDEX.json (kind file...)
  python - "$@" <<'PY'
import json, sys
kind, files = sys.argv[1], sys.argv[2:]
p = "profiles/INDEX.json"
d = json.load(open(p))
d[kind] = files + [f for f in d.get(kind, []) if f not in files]
json.dump(d, open(p, "w"), indent=1)
PY
  cp profiles/INDEX.json $OUT/
}
rocprof_stats() {   # NAME cfg size nary bench-args...
  local NAME=$1 CF=$2 SZ=$3 NA=$4; shift 4
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${NAME}_prof -o run --output-format csv -- python bench.py --no-cpu "$@" > gpurun_out/${NAME}_rocprof_bench.log 2>&1 || { tail -5 gpurun_out/${NAME}_rocprof_bench.log; return 1; }
  local ST=$(ls gpurun_out/${NAME}_prof/*/run_kernel_stats.csv gpurun_out/${NAME}_prof/run_kernel_stats.csv 2>/dev/null | head -1)
  cp $ST $OUT/${NAME}_kernel_stats.csv && python tools/rocprof_report.py $ST $OUT/${NAME}_rocprof.json $CF $SZ $NA > /dev/null || return 1
  cp $OUT/${NAME}_rocprof.json profiles/
}
pmc_traffic() {   # NAME cfg size nary bench-args...
  local NAME=$1 CF=$2 SZ=$3 NA=$4; shift 4
  local D=gpurun_out/${NAME}_pmc
  rm -rf $D; mkdir -p $D
  local i=0
  for PASS in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $PASS -d $D/p$i -o run --output-format csv -- python bench.py --no-cpu --steps 2 --warmup 1 --prewarm 2 --profile-steps 1 "$@" > $D/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $D/p$i.log; return 1; }
  done
  PMC_ALL=1 PMC_KEEP_TEMPLATE=${KEEP_TEMPLATE:-} python tools/pmc_report.py $D $OUT/${NAME}_pmc_traffic.json $CF $SZ $NA > $OUT/${NAME}_pmc.txt || return 1
  cp $OUT/${NAME}_pmc_traffic.json profiles/
}
brief() { python tools/bench_brief.py; }
# ---- profiles first (so the bench lines below cite them)
rocprof_stats ${TAG} C2 $GiB 2 || exit 1
pmc_traffic ${TAG} C2 $GiB 2 || exit 1
rocprof_stats ${TAG}_C3 C3 $GiB 16 --cfg C3 --nary 16 || exit 1
pmc_traffic ${TAG}_C3 C3 $GiB 16 --cfg C3 --nary 16 || exit 1
rocprof_stats ${TAG}_C4 C4 $GiB 2 --cfg C4 --nary 2 || exit 1
pmc_traffic ${TAG}_C4 C4 $GiB 2 --cfg C4 --nary 2 || exit 1
rocprof_stats ${TAG}_C5 C5 $GiB 16 --cfg C5 --nary 16 --frontend || exit 1
pmc_traffic ${TAG}_C5 C5 $GiB 16 --cfg C5 --nary 16 --frontend || exit 1
index_add rocprof ${TAG}_rocprof.json ${TAG}_C3_rocprof.json ${TAG}_C4_rocprof.json ${TAG}_C5_rocprof.json
index_add pmc_traffic ${TAG}_pmc_traffic.json ${TAG}_C3_pmc_traffic.json ${TAG}_C4_pmc_traffic.json ${TAG}_C5_pmc_traffic.json
echo "profiles done"
# ---- the bench lines
timeout -k 10 400 python bench.py > $OUT/${TAG}_bench.log 2>&1 || { tail -5 $OUT/${TAG}_bench.log; exit 1; }
tail -1 $OUT/${TAG}_bench.log | brief
for cfg in "C3 16" "C4 2" "C5 16 --frontend" "C5 16 --frontend --two-stage"; do
  set -- $cfg
  name=$(echo "$cfg" | tr -d ' -' )
  timeout -k 10 300 python bench.py --no-cpu --cfg $1 --nary $2 ${@:3} > $OUT/${TAG}_cfg_${name}.log 2>&1 || { tail -5 $OUT/${TAG}_cfg_${name}.log; exit 1; }
  tail -1 $OUT/${TAG}_cfg_${name}.log | brief
done
# ---- nybble: PMC traffic (static, adaptive), then the lines with their CPU baselines and rocprof
for m in static adaptive; do
  KEEP_TEMPLATE=1 pmc_traffic ${TAG}_nyb_$m C1-nyb-$m $GiB 0 --codec nybble --mode $m || exit 1
done
index_add pmc_traffic ${TAG}_pmc_traffic.json ${TAG}_C3_pmc_traffic.json ${TAG}_C4_pmc_traffic.json ${TAG}_C5_pmc_traffic.json ${TAG}_nyb_static_pmc_traffic.json ${TAG}_nyb_adaptive_pmc_traffic.json
for m in static adaptive; do
  timeout -k 10 400 python bench.py --codec nybble --mode $m > $OUT/${TAG}_nyb_$m.log 2>&1 || { tail -5 $OUT/${TAG}_nyb_$m.log; exit 1; }
  tail -1 $OUT/${TAG}_nyb_$m.log | brief
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_nprof_$m -o run --output-format csv -- python bench.py --codec nybble --mode $m --no-cpu > gpurun_out/${TAG}_nyb_${m}_rocprof.log 2>&1 || { tail -5 gpurun_out/${TAG}_nyb_${m}_rocprof.log; exit 1; }
  ST=$(ls gpurun_out/${TAG}_nprof_$m/*/run_kernel_stats.csv gpurun_out/${TAG}_nprof_$m/run_kernel_stats.csv 2>/dev/null | head -1)
  cp $ST $OUT/${TAG}_nyb_${m}_kernel_stats.csv
done
echo "profile6 done"
