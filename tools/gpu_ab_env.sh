# Same-box A/B of an environment knob on the bench line: for each setting, bench.py --no-cpu
# (interleaved twice), after optional GPU tests selected by -k.
# usage: bash tools/gpu_ab_env.sh TAG VAR "v1 v2" "pytest -k expr|-" [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; VAR=$2; VALS=$3; K=$4; shift 4
mkdir -p gpurun_out
if [ "$K" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/${TAG}_tests.log | head -20; tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
for rep in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python bench.py --no-cpu "$@" > gpurun_out/${TAG}_${VAR}${v}_$rep.log 2>&1 || { tail -5 gpurun_out/${TAG}_${VAR}${v}_$rep.log; exit 1; }
    echo "$VAR=$v rep $rep: $(tail -1 gpurun_out/${TAG}_${VAR}${v}_$rep.log | python tools/bench_brief.py | tr '\n' ' ')"
  done
done
