# same-box A/B of the nybble static writers: in-tree library vs tools/_ablH (before the r3 writer rewrite)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for lib in tree ablH; do
    if [ $lib = tree ]; then unset DC_CORE_LIB; else export DC_CORE_LIB=$PWD/tools/_ablH/libdc_core.so; fi
    timeout -k 10 300 python bench.py --codec nybble --mode static --no-cpu > gpurun_out/r3n_$lib.log 2>&1 || { tail -5 gpurun_out/r3n_$lib.log; exit 1; }
    tail -1 gpurun_out/r3n_$lib.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], {k:v.get('ms') for k,v in d['kernels'].items()})"
  done
done
