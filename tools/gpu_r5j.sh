# pack variant with masked stage ORs and merged quarters (DC_OPT_PACK_QEMIT): parity, A/B on
# the C2 and C4 encode (k_huff_pack), then the round profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r5j}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "pack" > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_ab.log
for r in 1 2 3; do
  for cfg in "C2 2" "C4 2"; do
    set -- $cfg
    for v in 0 1; do
      timeout -k 10 150 python tools/abl_time.py --stage encode --cfg $1 --nary $2 --iters 10 --warm 10 --opt pack_qemit=$v --tag qemit=$v >> gpurun_out/${T}_ab.log 2>&1 || { tail -3 gpurun_out/${T}_ab.log; exit 1; }
    done
  done
done
grep '^{' gpurun_out/${T}_ab.log | cut -c1-300
