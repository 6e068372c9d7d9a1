# Steps in flight in bench.py (--in-flight): C2 (1 vs 2 vs 3), C3, C4, C5 fused and two stages,
# then the 2-rank gloo rehearsal of C2 and fused C5 (one host thread, lanes interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=r5u
line() {   # NAME args...
  local NAME=$1; shift
  timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/${T}_${NAME}.log 2>&1 || { tail -5 gpurun_out/${T}_${NAME}.log; return 1; }
  echo "== $NAME"; tail -1 gpurun_out/${T}_${NAME}.log | python tools/bench_brief.py
}
line C2_f2 && line C2_f1 --in-flight 1 && line C2_f3 --in-flight 3 && line C3 --cfg C3 --nary 16 && line C4 --cfg C4 --nary 2 \
  && line C5 --cfg C5 --nary 16 --frontend && line C5_two --cfg C5 --nary 16 --frontend --two-stage || exit 1
for cfg in "C2 2" "C5 16 --frontend"; do
  set -- $cfg
  name=$(echo "$cfg" | tr -d ' -')
  DC_BENCH_BACKEND=gloo timeout -k 10 280 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 --prewarm 5 --no-cpu --cfg $1 --nary $2 ${@:3} > gpurun_out/${T}_gloo2_${name}.log 2>&1 || { tail -8 gpurun_out/${T}_gloo2_${name}.log; exit 1; }
  echo "== gloo2 $name"; grep -E '^\{' gpurun_out/${T}_gloo2_${name}.log | python tools/bench_brief.py
done
