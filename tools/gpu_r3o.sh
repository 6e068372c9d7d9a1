# adaptive nybble encode: MTF walk with deeper prefetch (tests + same-box A/B against tools/_ablH)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "nyb" > gpurun_out/r3o_nyb_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/r3o_nyb_tests.log | head -20; tail -3 gpurun_out/r3o_nyb_tests.log; exit 1; }
tail -1 gpurun_out/r3o_nyb_tests.log
for r in 1 2; do
  for lib in tree ablH; do
    if [ $lib = tree ]; then unset DC_CORE_LIB; else export DC_CORE_LIB=$PWD/tools/_ablH/libdc_core.so; fi
    timeout -k 10 300 python bench.py --codec nybble --mode adaptive --no-cpu > gpurun_out/r3o_$lib.log 2>&1 || { tail -5 gpurun_out/r3o_$lib.log; exit 1; }
    tail -1 gpurun_out/r3o_$lib.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['roofline']['frac'], {k:v.get('ms') for k,v in d['kernels'].items()}, d['decode_sample']['MBps'])"
  done
done
