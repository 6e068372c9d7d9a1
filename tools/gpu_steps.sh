# bench.py ms_per_step against --steps (the driver runs --steps 20 --warmup 5): fixed cost of
# the timed region = (ms(K) - ms(inf)) * K
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for k in 5 20 50 200; do
  timeout -k 10 300 python bench.py --steps $k --warmup 5 --no-cpu > gpurun_out/steps_$k.log 2>&1 || { tail -5 gpurun_out/steps_$k.log; exit 1; }
  tail -1 gpurun_out/steps_$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('steps', $k, 'ms', d['ms_per_step'], 'GBps', d['value'])"
done
