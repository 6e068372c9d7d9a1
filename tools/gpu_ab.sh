# A/B of a context option on one stage (run under gpurun): bash tools/gpu_ab.sh STAGE OPTION VALUES [CFG] [TESTS-K]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -n "$5" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "$5" > gpurun_out/ab_tests.log 2>&1 || { grep -E "^E|Error|assert" gpurun_out/ab_tests.log | head -20; tail -5 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
timeout -k 10 300 python -u tools/kern_ab.py --stage $1 --option $2 --values $3 --cfg ${4:-C2}
