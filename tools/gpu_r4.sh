# Round-4 GPU call: [tests] -> bench line (-> optional extra bench args). Logs under gpurun_out/.
# usage: bash tools/gpu_r4.sh TAG [tests|notests] [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r4x}; MODE=${2:-tests}; shift 2 2>/dev/null
mkdir -p gpurun_out
if [ "$MODE" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|error" gpurun_out/${TAG}_gpu_tests.log | head -20; tail -5 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_gpu_tests.log
fi
timeout -k 10 300 python bench.py "$@" > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | python tools/bench_brief.py
