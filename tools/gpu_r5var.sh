# Run-to-run spread of the default bench line on one box: three runs back to back
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r5var_$i.log 2>&1 || { tail -5 gpurun_out/r5var_$i.log; exit 1; }
  echo "run $i: $(tail -1 gpurun_out/r5var_$i.log | python tools/bench_brief.py | head -1)"
done
