# nybble static writers: in-tree (entry/loc loads hoisted) vs tools/_ablW/libdc_core_base.so (HEAD)
# vs tools/_ablN (element loop ablated)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for lib in tree base ablN tree base; do
  case $lib in tree) unset DC_CORE_LIB;; base) export DC_CORE_LIB=$PWD/tools/_ablW/libdc_core_base.so;; ablN) export DC_CORE_LIB=$PWD/tools/_ablN/libdc_core.so;; esac
  timeout -k 10 300 python bench.py --codec nybble --mode static --no-cpu > gpurun_out/r3u_$lib.log 2>&1
  tail -1 gpurun_out/r3u_$lib.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', {k:v.get('ms') for k,v in d['kernels'].items()})" || tail -3 gpurun_out/r3u_$lib.log
done
