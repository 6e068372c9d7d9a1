# decoder variants: parity tests then A/B (run under gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "decode or pack_bit or full_size or sharded_huffman or offset" > gpurun_out/dec9_tests.log 2>&1
rc=$?
tail -5 gpurun_out/dec9_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/kern_ab.py --stage decode --option decode_variant --values 0,1,3 > gpurun_out/dec9_ab.log 2>&1
rc=$?
tail -4 gpurun_out/dec9_ab.log
exit $rc
