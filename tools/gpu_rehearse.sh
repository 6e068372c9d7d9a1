# Multi-rank rehearsal on a one-GPU box (run under gpurun): ranks share the GPU, collectives over
# gloo (RCCL refuses two ranks on one device). 2-rank C2 (broadcast table default, gather timed),
# then 4-rank C2 with the input generated on the device, 4-rank fused C5 and 3-rank C4 (the r2/r3 stall of 4 processes' torch
# generation at once is gone with synth.device_text's flat gather), per-rank phase lines and
# stack dumps. Prints each line's value, the launches per step of every kernel, round trip.
# usage: bash tools/gpu_rehearse.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r4x}
mkdir -p gpurun_out
run() {   # N PORT LOG extra-args...
  local N=$1 P=$2 LOG=$3; shift 3
  DC_BENCH_BACKEND=gloo DC_BENCH_PHASES=1 DC_BENCH_TRACE_AFTER=30 timeout -k 10 280 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port $P bench.py --gpus $N --steps 5 --warmup 2 --prewarm 5 --no-cpu "$@" > $LOG 2>&1
  local rc=$?
  grep -E '^\{' $LOG | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('N', d['n_gpus'], 'value', d['value'], 'ms', d['ms_per_step'], 'table', d.get('table_mode'), 'launches/step', sum(v['launches_per_step'] for v in k.values()), {n: v['launches_per_step'] for n, v in k.items()}, 'gather', d.get('gather'), 'ok', d['roundtrip_ok'])" || true
  grep -E "rank [0-9]\]" $LOG | tail -8
  return $rc
}
run 2 29511 gpurun_out/${TAG}_gloo2_C2.log --gather-reps 1 || exit 1
run 2 29513 gpurun_out/${TAG}_gloo2_C2_replicate.log --gather-reps 0 --table-mode replicate || exit 1
run 4 29512 gpurun_out/${TAG}_gloo4_C2_devsynth.log --gather-reps 1 || { for f in gpurun_out/trace_rank*.log; do echo "== $f"; tail -12 $f; done; exit 1; }
run 4 29514 gpurun_out/${TAG}_gloo4_C5_fused.log --cfg C5 --nary 16 --frontend || exit 1
run 3 29515 gpurun_out/${TAG}_gloo3_C4.log --cfg C4 --nary 2 --gather-reps 1 || exit 1
