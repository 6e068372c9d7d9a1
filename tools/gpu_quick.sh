# quick GPU check (run under gpurun): pack/decode parity tests, then one bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t1.log 2>&1
rc=$?
tail -15 gpurun_out/t1.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/b1.log 2>&1
rc=$?
tail -1 gpurun_out/b1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()})"
exit $rc
