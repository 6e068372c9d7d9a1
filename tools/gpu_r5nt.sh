# Persistent k_nyb_tiles (working tree at the time, not committed: see profiles/r5nt_nyb_tiles_persistent_ab.log) (the next tile pair's loads in flight) against the last commit's
# library (tools/_old), nybble static step, interleaved; nybble GPU tests first
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "nybble or nyb" > gpurun_out/r5nt_tests.log 2>&1 || { tail -20 gpurun_out/r5nt_tests.log; exit 1; }
tail -1 gpurun_out/r5nt_tests.log
bash tools/gpu_ab_old.sh r5nt "nyb_static_step C1 0" "nyb_adaptive C1 0"
