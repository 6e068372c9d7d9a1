# Round-5 call r: fused C5 step probe (host time per step), the edge-load A/B (C5 encode), C5 tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python tools/c5_step_probe.py > gpurun_out/r5r_c5probe.log 2>&1 || { tail -3 gpurun_out/r5r_c5probe.log; exit 1; }
tail -2 gpurun_out/r5r_c5probe.log | cut -c1-700
bash tools/gpu_ab_old.sh r5r "c5_enc C5 16" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_c5_shards.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "c5 or small or fe_ or fused or shard" > gpurun_out/r5r_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/r5r_tests.log | head -20; exit 1; }
tail -1 gpurun_out/r5r_tests.log
