# decode redo with the groups' first starts beside the masks: decode tests + same-box A/B (C2, C5)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "decode or huff or fullsize or dist or shard" > gpurun_out/r3q_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/r3q_tests.log | head -20; tail -3 gpurun_out/r3q_tests.log; exit 1; }
tail -1 gpurun_out/r3q_tests.log
echo "tree:"; timeout -k 10 200 python -u tools/kern_ab.py --stage decode --option decode_static_pct --values 60 --cfg C2 --nary 2 --rounds 3 || exit 1
echo "ablH:"; DC_CORE_LIB=$PWD/tools/_ablH/libdc_core.so timeout -k 10 200 python -u tools/kern_ab.py --stage decode --option decode_static_pct --values 60 --cfg C2 --nary 2 --rounds 3 || exit 1
echo "tree:"; timeout -k 10 200 python -u tools/kern_ab.py --stage decode --option decode_static_pct --values 60 --cfg C2 --nary 2 --rounds 3 || exit 1
echo "ablH:"; DC_CORE_LIB=$PWD/tools/_ablH/libdc_core.so timeout -k 10 200 python -u tools/kern_ab.py --stage decode --option decode_static_pct --values 60 --cfg C2 --nary 2 --rounds 3 || exit 1
