# Round-5: the one-lane-per-stream nybble kernels (DCNK, batch decode) with staged lane IO:
# their GPU tests, then the adaptive bench line (decode_batch) and a PMC pass over the batch decode.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-nyblane}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread -k "nyb or nybble or chunked or batch" > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_tests.log | head -20; tail -3 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
[ -n "$SKIP_BENCH" ] || timeout -k 10 300 python bench.py --codec nybble --mode adaptive --no-cpu > gpurun_out/${TAG}_adaptive.log 2>&1 || { tail -5 gpurun_out/${TAG}_adaptive.log; exit 1; }
[ -n "$SKIP_BENCH" ] || tail -1 gpurun_out/${TAG}_adaptive.log | cut -c1-1500
for st in batch chunk_enc; do
  timeout -k 10 120 python tools/abl_time.py --stage $st --cfg C1 --iters 5 --warm 3 >> gpurun_out/${TAG}_abl.log 2>&1 || { tail -3 gpurun_out/${TAG}_abl.log; exit 1; }
done
grep '^{' gpurun_out/${TAG}_abl.log
for st in batch chunk_enc; do
  DC_CORE_LIB=tools/_old/libdc_core.so timeout -k 10 120 python tools/abl_time.py --stage $st --cfg C1 --iters 5 --warm 3 >> gpurun_out/${TAG}_abl_old.log 2>&1 || { tail -3 gpurun_out/${TAG}_abl_old.log; exit 1; }
done
grep '^{' gpurun_out/${TAG}_abl_old.log
