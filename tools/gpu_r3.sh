# Round-3 GPU call (run under gpurun): bash tools/gpu_r3.sh TAG "pytest -k expr" "ablation dirs" [stage]
#   1. selected GPU tests   2. same-box A/B of one stage: in-tree library vs tools/_abl<X>
#   3. bench line (C2 default)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3}; K=${2:-decode}; ABL=${3:-}; STAGE=${4:-decode}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -k "$K" --timeout 100 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; grep -cE "PASSED" gpurun_out/${TAG}_tests.log; tail -2 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit $rc; fi
for r in 1 2; do
  echo "base:"; timeout -k 10 200 python -u tools/kern_ab.py --stage $STAGE --option decode_static_pct --values 60 --cfg C2 --rounds 3 || exit 1
  for x in $ABL; do
    echo "abl$x:"; DC_CORE_LIB=$PWD/tools/_abl$x/libdc_core.so timeout -k 10 200 python -u tools/kern_ab.py --stage $STAGE --option decode_static_pct --values 60 --cfg C2 --rounds 3 || exit 1
  done
done
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'enc', r['encode_ms'], r['encode_frac'], 'dec', r['decode_ms'], r['decode_frac'], 'ok', d['roundtrip_ok'], {k: v['ms'] for k, v in d['kernels'].items()})"
