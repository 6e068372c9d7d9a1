# Nybble PMC traffic (FETCH_SIZE x2 + WRITE_SIZE per launch, MI355X_MICROARCH.md § HBM) of the
# static and adaptive bench lines, one counter group per rocprofv3 pass: profiles JSON that
# bench.py's nybble lines read as roofline.traffic. usage: bash tools/gpu_nyb_pmc.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r4n}
mkdir -p gpurun_out profiles
N=1073741824   # bench.py --size default (1 GiB)
for m in static adaptive; do
  O=gpurun_out/${TAG}_nybpmc_$m
  rm -rf $O; mkdir -p $O
  i=0
  for PASS in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $PASS -d $O/p$i -o run --output-format csv -- python bench.py --codec nybble --mode $m --no-cpu --steps 2 --warmup 1 --profile-steps 1 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  done
  PMC_ALL=1 PMC_KEEP_TEMPLATE=1 python tools/pmc_report.py $O gpurun_out/${TAG}_nyb_${m}_pmc_traffic.json C1-nyb-$m $N 0 > gpurun_out/${TAG}_nyb_${m}_pmc.txt || exit 1
  cp gpurun_out/${TAG}_nyb_${m}_pmc_traffic.json profiles/
  grep -A3 "k_fsm_write<0>\|k_fsm_write<1>\|k_mtf_walk" gpurun_out/${TAG}_nyb_${m}_pmc.txt | head -30
done
