# Same-box A/B of context-option kernel variants in the A/B build (tools/_ab: diag_build.sh _ab
# -DDC_AB_KERNELS): each variant's stream checked against the default kernels' (variant_check.py),
# then per-kernel HIP-event times (abl_time.py), interleaved rounds.
#   gpurun -- bash tools/gpu_ab.sh TAG STAGE "cfg nary" "opt=v ..." ["opt=v ..."]...
#   (an empty option string "" is the default kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; ST=$2; CN=$3; shift 3
read -r CF NA <<< "$CN"
mkdir -p gpurun_out
L=gpurun_out/${TAG}_ab.log
: > $L
export DC_CORE_LIB=$PWD/tools/${AB_LIB:-_ab}/libdc_core.so
for V in "$@"; do
  [ -z "$V" ] && continue
  O=""; for kv in $V; do O="$O --opt $kv"; done
  timeout -k 10 120 python tools/variant_check.py --cfg $CF --nary $NA $O >> $L 2>&1 || { grep -v amdgpu.ids $L | tail -3; exit 1; }
done
for r in 1 2; do
  for V in "$@"; do
    O=""; for kv in $V; do O="$O --opt $kv"; done
    timeout -k 10 150 python tools/abl_time.py --stage $ST --cfg $CF --nary $NA --iters 20 --warm 20 --tag "[$V]" $O >> $L 2>&1 || { grep -v amdgpu.ids $L | tail -3; exit 1; }
  done
done
grep -v amdgpu.ids $L | cut -c1-300
