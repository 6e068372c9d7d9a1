# Adaptive nybble encode writer a wave per tile (k_nyb_enc_wtile<true>) vs k_fsm_write: nybble
# tests, same-process A/B of the adaptive encode
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r5z2}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "nybble" > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_ab.log
for r in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 150 python tools/abl_time.py --stage nyb_adaptive --cfg C1 --nary 0 --iters 10 --warm 10 --opt nyb_wtile_off=$v --tag wtile_off=$v >> gpurun_out/${T}_ab.log 2>&1 || { tail -3 gpurun_out/${T}_ab.log; exit 1; }
  done
done
grep '^{' gpurun_out/${T}_ab.log | cut -c1-400
