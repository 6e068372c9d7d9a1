# BASELINE configs C3-C5 on one GPU (bench.py options; the default bench line is C2)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/cfg_$tag.log 2>&1 || { tail -5 gpurun_out/cfg_$tag.log; exit 1; }
  tail -1 gpurun_out/cfg_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['encode_GBps'], d['decode_GBps'], d['ratio'], d['roundtrip_ok'], d['roofline']['kernel'], d['roofline']['frac'])"; }
run C3 --cfg C3 --nary 16
run C4 --cfg C4 --nary 2
run C5 --cfg C5 --nary 16 --frontend
