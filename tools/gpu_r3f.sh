# round-3 call (run under gpurun): GPU tests, bench, decode A/B vs the r2 library, copy probe shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3f}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -cE "PASSED" gpurun_out/${TAG}_tests.log; tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'enc', r.get('encode_ms'), r.get('encode_frac'), 'dec', r.get('decode_ms'), r.get('decode_frac'), 'copy', r.get('copy_probe_GBps'), r.get('frac_vs_copy'), 'ok', d['roundtrip_ok'], {k: v['ms'] for k, v in d['kernels'].items()})"
for cfg in C2 C4; do
  for r in 1 2; do
    echo "$cfg now:"; timeout -k 10 200 python -u tools/kern_ab.py --stage decode --option decode_static_pct --values 60 --cfg $cfg --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
    echo "$cfg r2:"; DC_CORE_LIB=$PWD/tools/_r2/libdc_core.so timeout -k 10 200 python -u tools/kern_ab.py --stage decode --option decode_static_pct --values 60 --cfg $cfg --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
timeout -k 10 120 tools/_copy_probe | tee gpurun_out/${TAG}_copy_probe.log
