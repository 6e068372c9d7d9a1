# nybble (+ RCCL) GPU tests, then the static and adaptive nybble bench lines.
# usage: bash tools/gpu_nyb.sh TAG [pytest -k expr]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r4x}; K=${2:-nybble or rccl}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/${TAG}_tests.log | head -20; tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for m in static adaptive; do
  timeout -k 10 300 python bench.py --codec nybble --mode $m --no-cpu > gpurun_out/${TAG}_nyb_$m.log 2>&1 || { tail -5 gpurun_out/${TAG}_nyb_$m.log; exit 1; }
  tail -1 gpurun_out/${TAG}_nyb_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$m', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('encode_frac'), r.get('decode_frac'), d.get('decode_sample'), d['roundtrip_ok']); print({k: v['ms'] for k, v in d['kernels'].items()})"
done
