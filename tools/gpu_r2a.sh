# round-2 baseline check (run under gpurun): all GPU tests, then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2a_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r2a_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/r2a_bench.log 2>&1 || { tail -5 gpurun_out/r2a_bench.log; exit 1; }
tail -1 gpurun_out/r2a_bench.log
