# Round-5 call f: pack A/B (k_huff_pack_w ranges of 1 block, G=4 forced) and the 3-deep histogram prefetch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r5f}
mkdir -p gpurun_out
L=gpurun_out/${TAG}_abl.log
: > $L
run() { timeout -k 10 120 python tools/abl_time.py --stage encode "$@" >> $L 2>&1 || { tail -3 $L; exit 1; }; }
for r in 1 2; do
  run --opt pack_block=1
  run --opt pack_grid=1
  run --opt pack_block=2 --opt pack_grid=1
  run --opt pack_block=2 --opt pack_grid=2
  run --opt pack_block=1 --opt hist_prefetch=3
done
grep '^{' $L
