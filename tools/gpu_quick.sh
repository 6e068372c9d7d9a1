set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "decode or pack_bit_exact or pack_at_bit" > gpurun_out/t1.log 2>&1
rc=$?
tail -30 gpurun_out/t1.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/b1.log 2>&1
rc=$?
tail -3 gpurun_out/b1.log
exit $rc
