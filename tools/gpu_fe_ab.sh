# same-box A/B of the C5 front-end + Huffman step: in-tree library vs tools/_abl<X> libraries
#   bash tools/gpu_fe_ab.sh "S"
set -o pipefail
cd $GRAFT_REPO_ROOT
one() {
  timeout -k 10 200 python bench.py --no-cpu --frontend --cfg C5 --nary 16 > gpurun_out/fe_ab.tmp 2>&1 || { tail -5 gpurun_out/fe_ab.tmp; exit 1; }
  tail -1 gpurun_out/fe_ab.tmp | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step'], 'ok', d['roundtrip_ok'], {k: v['ms'] for k, v in d['kernels'].items() if k.startswith('small')})"
}
for r in 1 2; do
  echo "tree:"; one
  for x in $1; do echo "abl$x:"; DC_CORE_LIB=$PWD/tools/_abl$x/libdc_core.so one; done
done
