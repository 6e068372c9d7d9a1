# Partial redo (DC_OPT_DECODE_PARTIAL_REDO, in the working tree at the time, not committed: the
# profiles/r5pr_partial_redo_ab.log header says what it was) tests and same-box A/B (C2 decode, C5 step), then
# steps in flight 2/3 on the C2 line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/r5pr_ab.log
: > $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "partial_redo or rare_codes or v8_equals or stale" tests/test_gpu_fe.py > gpurun_out/r5pr_tests.log 2>&1 || { tail -20 gpurun_out/r5pr_tests.log; exit 1; }
tail -1 gpurun_out/r5pr_tests.log
for r in 1 2; do
  for v in 1 2; do
    timeout -k 10 150 python tools/abl_time.py --stage decode --cfg C2 --nary 2 --iters 10 --warm 10 --opt decode_partial_redo=$v --tag C2_pr$v >> $L 2>&1 || { tail -3 $L; exit 1; }
    timeout -k 10 150 python tools/abl_time.py --stage c5_step --cfg C5 --nary 16 --iters 10 --warm 10 --opt decode_partial_redo=$v --tag C5_pr$v >> $L 2>&1 || { tail -3 $L; exit 1; }
  done
done
grep '^{' $L | cut -c1-400
for L2 in 2 3; do
  timeout -k 10 200 python bench.py --no-cpu --in-flight $L2 > gpurun_out/r5if_$L2.log 2>&1 || { tail -5 gpurun_out/r5if_$L2.log; exit 1; }
  echo "in_flight $L2: $(tail -1 gpurun_out/r5if_$L2.log | python tools/bench_brief.py | head -1)"
done
