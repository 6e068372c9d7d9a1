# Same-box timing of ablation libraries (tools/<dir>/libdc_core.so, garbage output: nothing is
# checked) against the tree's, per-kernel HIP-event times. usage: bash tools/gpu_abl_lib.sh TAG "stage cfg nary" dir...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; SPEC=$2; shift 2
read -r ST CF NA <<< "$SPEC"
mkdir -p gpurun_out
L=gpurun_out/${TAG}_abl.log
: > $L
for r in 1 2; do
  timeout -k 10 150 python tools/abl_time.py --stage $ST --cfg $CF --nary $NA --iters 10 --warm 10 --tag base >> $L 2>&1 || { tail -3 $L; exit 1; }
  for d in "$@"; do
    DC_CORE_LIB=tools/$d/libdc_core.so timeout -k 10 150 python tools/abl_time.py --stage $ST --cfg $CF --nary $NA --iters 10 --warm 10 --tag $d >> $L 2>&1 || { tail -3 $L; exit 1; }
  done
done
grep '^{' $L | cut -c1-400
