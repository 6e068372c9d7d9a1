# A/B of an environment knob on the default bench line: VAR=name VALUES="a b c" bash tools/ab_env.sh
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in $VALUES; do
  env $VAR=$v timeout -k 10 200 python bench.py --no-cpu > gpurun_out/abe_$v.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/abe_$v.log; exit 1; }
  tail -1 gpurun_out/abe_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$v', d['value'], d['ms_per_step'], d['kernels']['huff_pack']['ms'], d['roundtrip_ok'])"
done
