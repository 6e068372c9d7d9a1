# adaptive decode: new resolve path (debug probe, tests, nybble adaptive bench line)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/dbg_adec.py 0 && timeout -k 10 120 python tools/dbg_adec.py 3 && timeout -k 10 200 python tools/dbg_adec2.py || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "nyb" > gpurun_out/r3m_nyb_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/r3m_nyb_tests.log | head -20; tail -3 gpurun_out/r3m_nyb_tests.log; exit 1; }
tail -1 gpurun_out/r3m_nyb_tests.log
timeout -k 10 300 python bench.py --codec nybble --mode adaptive > gpurun_out/r3m_nyb_adaptive.log 2>&1 || { tail -5 gpurun_out/r3m_nyb_adaptive.log; exit 1; }
tail -1 gpurun_out/r3m_nyb_adaptive.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['decode_sample'], d['roundtrip_ok'], d['value'])"
timeout -k 10 300 python bench.py --codec nybble --mode static > gpurun_out/r3m_nyb_static.log 2>&1 || { tail -5 gpurun_out/r3m_nyb_static.log; exit 1; }
tail -1 gpurun_out/r3m_nyb_static.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('static', d['value'], r['frac'], r.get('encode_frac'), r.get('decode_frac'), {k:v.get('ms') for k,v in d['kernels'].items()}, d['roundtrip_ok'])"
