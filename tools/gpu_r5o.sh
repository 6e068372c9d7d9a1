# Round-5 call o: the fused C5 encode of shards (world > 1): its GPU parity tests (one context per
# simulated rank), the C5 GPU tests at world 1, then the 2-rank gloo rehearsal of the C5 line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r5o}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_c5_shards.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "c5 or small or fe_ or fused or shard" > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_tests.log | head -20; tail -3 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
LOG=gpurun_out/${TAG}_gloo2_C5_fused.log
DC_BENCH_BACKEND=gloo DC_BENCH_PHASES=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 5 --warmup 2 --prewarm 5 --no-cpu --cfg C5 --frontend --nary 16 --size 268435456 > $LOG 2>&1 || { tail -20 $LOG; exit 1; }
grep -E '^\{' $LOG | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('N', d['n_gpus'], 'value', d['value'], 'ms', d['ms_per_step'], 'launches/step', sum(v['launches_per_step'] for v in k.values()), {n: v['launches_per_step'] for n, v in k.items()}, 'ok', d['roundtrip_ok'])"
