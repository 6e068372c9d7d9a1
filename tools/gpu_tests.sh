# run selected GPU tests (run under gpurun): bash tools/gpu_tests.sh TAG "pytest args"
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}.log | tail -25
exit $rc
