# Round-5 call m: the round-end checks after the diagnostic strip, then the per-lane nybble timings.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_verify.sh ${1:-r5m} || exit 1
SKIP_BENCH= bash tools/gpu_nyb_lane.sh ${1:-r5m}_nyb
