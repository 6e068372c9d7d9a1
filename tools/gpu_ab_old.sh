# Same-box A/B of the tree's library against tools/_old (the last commit's), per-kernel HIP-event
# times (tools/abl_time.py), interleaved rounds. usage: bash tools/gpu_ab_old.sh TAG "stage cfg nary" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
L=gpurun_out/${TAG}_ab.log
: > $L
SPECS=("$@")
for r in 1 2; do
  for spec in "${SPECS[@]}"; do
    read -r ST CF NA <<< "$spec"
    timeout -k 10 150 python tools/abl_time.py --stage $ST --cfg $CF --nary $NA --iters 10 --warm 10 --tag new >> $L 2>&1 || { tail -3 $L; exit 1; }
    DC_CORE_LIB=tools/_old/libdc_core.so timeout -k 10 150 python tools/abl_time.py --stage $ST --cfg $CF --nary $NA --iters 10 --warm 10 --tag old >> $L 2>&1 || { tail -3 $L; exit 1; }
  done
done
grep '^{' $L | cut -c1-400
