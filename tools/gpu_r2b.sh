# GPU tests + bench + rocprof kernel trace of the bench (run under gpurun): bash tools/gpu_r2b.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r2b}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_tests.log | head; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'enc', r['encode_ms'], r['encode_frac'], 'dec', r['decode_ms'], r['decode_frac'], {k: v['ms'] for k, v in d['kernels'].items()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/${TAG}_rocprof.log 2>&1 || { tail -5 gpurun_out/${TAG}_rocprof.log; exit 1; }
ls gpurun_out/${TAG}_prof
