# C5 check (under gpurun): the front-end / fused GPU tests, then the C5 line (fused).
# usage: bash tools/gpu_c5.sh TAG [two]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-c5}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread -k "small or fused or c5 or frontend or fallback or raw_high" > gpurun_out/${TAG}_c5_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/${TAG}_c5_tests.log | head -20; tail -5 gpurun_out/${TAG}_c5_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_c5_tests.log
timeout -k 10 300 python bench.py --no-cpu --frontend --cfg C5 --nary 16 > gpurun_out/${TAG}_C5.log 2>&1 || { tail -5 gpurun_out/${TAG}_C5.log; exit 1; }
tail -1 gpurun_out/${TAG}_C5.log | python tools/bench_brief.py
if [ -n "$2" ]; then
  timeout -k 10 300 python bench.py --no-cpu --frontend --cfg C5 --nary 16 --two-stage > gpurun_out/${TAG}_C5_two.log 2>&1 || { tail -5 gpurun_out/${TAG}_C5_two.log; exit 1; }
  tail -1 gpurun_out/${TAG}_C5_two.log | python tools/bench_brief.py
fi
