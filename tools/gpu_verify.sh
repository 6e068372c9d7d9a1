# The round-end checks on one box: every GPU test, smoke() and the default bench line.
#   gpurun -- bash tools/gpu_verify.sh TAG [--cpu]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-verify}
CPU=--no-cpu
[ "$2" = "--cpu" ] && CPU=
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_gpu_tests.log | head
tail -1 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py $CPU > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | python tools/bench_brief.py
