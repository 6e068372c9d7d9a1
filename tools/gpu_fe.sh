# C5 front-end bench + kernel trace (run under gpurun): bash tools/gpu_fe.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-fe}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu --frontend --cfg C5 --nary 16 > gpurun_out/${TAG}_fe_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_fe_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_fe_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('C5 value', d['value'], 'ms', d['ms_per_step'], 'ok', d['roundtrip_ok'], {k: v['ms'] for k, v in d['kernels'].items()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_fe_prof -o run --output-format csv -- python bench.py --no-cpu --frontend --cfg C5 --nary 16 --steps 3 --warmup 1 --profile-steps 1 > gpurun_out/${TAG}_fe_rocprof.log 2>&1 || { tail -5 gpurun_out/${TAG}_fe_rocprof.log; exit 1; }
