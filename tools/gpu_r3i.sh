# round-3 call (run under gpurun): GPU tests + bench, multi-rank rehearsals, torch-generation stall probe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3i}
mkdir -p gpurun_out
rm -f gpurun_out/trace_rank*.log
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -cE "PASSED" gpurun_out/${TAG}_tests.log; tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'enc', r.get('encode_ms'), r.get('encode_frac'), 'dec', r.get('decode_ms'), r.get('decode_frac'), 'ok', d['roundtrip_ok'], {k: v['ms'] for k, v in d['kernels'].items()})"
bash tools/gpu_rehearse.sh ${TAG} || exit 1
timeout -k 10 600 python -u tools/synth_stall.py 60 2>&1 | tee gpurun_out/${TAG}_synth_stall.log
