# k_mtf_resolve with its step records read 4 at a time (the next 4 in flight): nybble tests,
# A/B of the adaptive encode against tools/_old (the last commit's library)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r5l}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "nybble" > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
bash tools/gpu_ab_old.sh ${T} "nyb_adaptive C1 0" || exit 1
