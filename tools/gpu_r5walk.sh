# k_mtf_walk<2> with fewer VALU per element (byte permutes for the touched byte, the moved-byte mask
# as z ^ (z - 1) with a popcount rank, one v_bfe for the next context, no dword selects for an
# aligned input): nybble tests, then the adaptive encode A/B against tools/_old (the last commit's)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r5walk}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "nybble" > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
bash tools/gpu_ab_old.sh ${T} "nyb_adaptive C1 0" || exit 1
