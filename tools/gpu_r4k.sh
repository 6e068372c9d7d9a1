# Round-4 check call: every GPU test, the C5 line fused against two-stage, the C2 line, the
# nybble lines and their PMC traffic. usage: bash tools/gpu_r4k.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r4k}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/${TAG}_gpu_tests.log | head -20; tail -5 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
for v in fused two; do
  X=""; [ $v = two ] && X="--two-stage"
  timeout -k 10 300 python bench.py --no-cpu --frontend --cfg C5 --nary 16 $X > gpurun_out/${TAG}_C5_$v.log 2>&1 || { tail -5 gpurun_out/${TAG}_C5_$v.log; exit 1; }
  tail -1 gpurun_out/${TAG}_C5_$v.log | python tools/bench_brief.py
done
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${TAG}_C2.log 2>&1 || { tail -5 gpurun_out/${TAG}_C2.log; exit 1; }
tail -1 gpurun_out/${TAG}_C2.log | python tools/bench_brief.py
for m in static adaptive; do
  timeout -k 10 300 python bench.py --codec nybble --mode $m --no-cpu > gpurun_out/${TAG}_nyb_$m.log 2>&1 || { tail -5 gpurun_out/${TAG}_nyb_$m.log; exit 1; }
  tail -1 gpurun_out/${TAG}_nyb_$m.log | python tools/bench_brief.py
done
bash tools/gpu_nyb_pmc.sh $TAG
