# C5 fused front-end encode: its GPU tests, then its kernel times on 1 GiB (under gpurun).
# usage: bash tools/gpu_fe2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-fe2}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fe.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_fe_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_fe_tests.log | head -30; tail -5 gpurun_out/${TAG}_fe_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_fe_tests.log
timeout -k 10 300 python tools/fe_time.py 10 > gpurun_out/${TAG}_fe_time.log 2>&1 || { tail -5 gpurun_out/${TAG}_fe_time.log; exit 1; }
tail -1 gpurun_out/${TAG}_fe_time.log
