set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_helpers.py tests/test_container.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tbl_tests.log 2>&1 || { grep -E "^E|Error|assert" gpurun_out/tbl_tests.log | head -20; tail -5 gpurun_out/tbl_tests.log; exit 1; }
tail -1 gpurun_out/tbl_tests.log
timeout -k 10 200 python tools/diag_table.py 2>&1 | tail -1
