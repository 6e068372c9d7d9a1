# full-size bit-exact tests (run under gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 400 --timeout-method thread > gpurun_out/fullsize.log 2>&1
rc=$?
tail -8 gpurun_out/fullsize.log
exit $rc
