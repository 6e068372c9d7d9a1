# Multi-rank rehearsal on a one-GPU box (run under gpurun): ranks share the GPU, collectives over
# gloo (RCCL refuses two ranks on one device). 2-rank C2 (broadcast table default, gather timed),
# then the 4-rank C2 case that stalled in r2, with per-rank phase lines and stack dumps.
# usage: bash tools/gpu_rehearse.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3r}
mkdir -p gpurun_out
run() {   # N PORT LOG extra-args...
  local N=$1 P=$2 LOG=$3; shift 3
  DC_BENCH_BACKEND=gloo DC_BENCH_PHASES=1 DC_BENCH_TRACE_AFTER=30 timeout -k 10 280 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port $P bench.py --gpus $N --steps 5 --warmup 2 --no-cpu "$@" > $LOG 2>&1
  local rc=$?
  grep -E '^\{' $LOG | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N', d['n_gpus'], 'value', d['value'], 'ms', d['ms_per_step'], 'table', d.get('table_mode'), 'gather', d.get('gather'), 'ok', d['roundtrip_ok'])" || true
  grep -E "rank [0-9]\]" $LOG | tail -8
  return $rc
}
run 2 29511 gpurun_out/${TAG}_gloo2_C2.log --gather-reps 1 || exit 1
# 4 ranks: the input generated on the host (DC_BENCH_SYNTH=host): four processes' torch
# generation at once on one GPU stalled in r2/r3 (tools/synth_stall.py isolates it)
DC_BENCH_SYNTH=host run 4 29512 gpurun_out/${TAG}_gloo4_C2.log --gather-reps 1 || { for f in gpurun_out/trace_rank*.log; do echo "== $f"; tail -12 $f; done; exit 1; }
