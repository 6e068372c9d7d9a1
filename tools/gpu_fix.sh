set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "decode" > gpurun_out/fix_tests.log 2>&1 || { tail -5 gpurun_out/fix_tests.log; exit 1; }
tail -1 gpurun_out/fix_tests.log
timeout -k 10 200 python tools/diag_fix.py 2>&1 | tail -1
timeout -k 10 200 python tools/kern_ab.py --stage decode --option decode_variant --values 0 --rounds 3 2>&1 | tail -1
