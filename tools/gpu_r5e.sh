# Round-5 call e: the wave-per-range pack (k_huff_pack_w): GPU tests, A/B against k_huff_pack.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r5e}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "pack or fixed8 or decode_of or full_size or sharded_huffman" > gpurun_out/${TAG}_pack_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_pack_tests.log | head -20; tail -3 gpurun_out/${TAG}_pack_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_pack_tests.log
L=gpurun_out/${TAG}_abl.log
: > $L
for r in 1 2; do
  timeout -k 10 120 python tools/abl_time.py --stage encode >> $L 2>&1 || { tail -3 $L; exit 1; }
  timeout -k 10 120 python tools/abl_time.py --stage encode --opt pack_block=1 >> $L 2>&1 || { tail -3 $L; exit 1; }
done
for bpw in 2 4 16; do
  timeout -k 10 120 python tools/abl_time.py --stage encode --opt pack_grid=$bpw >> $L 2>&1 || { tail -3 $L; exit 1; }
done
timeout -k 10 120 python tools/abl_time.py --stage encode --cfg C4 >> $L 2>&1 || { tail -3 $L; exit 1; }
timeout -k 10 120 python tools/abl_time.py --stage encode --cfg C4 --opt pack_block=1 >> $L 2>&1 || { tail -3 $L; exit 1; }
grep '^{' $L
timeout -k 10 500 python -u -m pytest tests/ -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_gpu_tests.log | head; tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | python tools/bench_brief.py
