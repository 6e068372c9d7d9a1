# round-3 call (run under gpurun): GPU tests, nybble lines, then the narrowed generation-stall probe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3j}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -cE "PASSED" gpurun_out/${TAG}_tests.log; tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit $rc; fi
for m in static adaptive; do
  timeout -k 10 400 python bench.py --codec nybble --mode $m --no-cpu > gpurun_out/${TAG}_nyb_$m.log 2>&1 || { tail -5 gpurun_out/${TAG}_nyb_$m.log; exit 1; }
  tail -1 gpurun_out/${TAG}_nyb_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('nyb $m', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('encode_frac'), r.get('decode_frac'), d['roundtrip_ok'], {k: v['ms'] for k, v in d['kernels'].items()})"
done
timeout -k 10 400 python -u tools/synth_stall.py 60 ss,mask2d 2>&1 | tee gpurun_out/${TAG}_synth_stall2.log
