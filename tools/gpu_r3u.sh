# nybble static encode writer: element-loop ablation (tools/_ablN) against the tree
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for lib in tree ablN tree ablN; do
  if [ $lib = tree ]; then unset DC_CORE_LIB; else export DC_CORE_LIB=$PWD/tools/_ablN/libdc_core.so; fi
  timeout -k 10 300 python bench.py --codec nybble --mode static --no-cpu > gpurun_out/r3u_$lib.log 2>&1
  tail -1 gpurun_out/r3u_$lib.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', {k:v.get('ms') for k,v in d['kernels'].items()})" || tail -3 gpurun_out/r3u_$lib.log
done
