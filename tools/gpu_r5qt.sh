# Decoder output by DPP transposes (working tree at the time, not committed; profiles/r5qt_decode_dpp_out_ab.log) against the last commit's library
# (tools/_old): decode GPU tests, then same-box A/B of the C2 / C4 decode and the C5 step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_fe.py -k "decode or roundtrip or fullsize or 1gib or fused" > gpurun_out/r5qt_tests.log 2>&1 || { tail -20 gpurun_out/r5qt_tests.log; exit 1; }
tail -1 gpurun_out/r5qt_tests.log
bash tools/gpu_ab_old.sh r5qt "decode C2 2" "decode C4 2" "c5_step C5 16"
