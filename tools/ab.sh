set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in ${VARIANTS:-base pf pf4}; do
  if [ $v = base ]; then unset DC_CORE_LIB; else export DC_CORE_LIB=$PWD/tools/_$v/libdc_core.so; fi
  timeout -k 10 200 python bench.py --no-cpu > gpurun_out/ab_$v.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/ab_$v.log; exit 1; }
  tail -1 gpurun_out/ab_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['kernels']['huff_pack']['ms'])"
done
