# Round-5 call b: the one-wave table merge + bitmap canonical codes: table/tree parity tests,
# table phase cycles (DC_DIAG build), decode per-wave split, bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r5b}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_helpers.py -m gpu -x -v --timeout 200 --timeout-method thread -k "table or huffman or tree or canonical or lengths or kat or golden" > gpurun_out/${TAG}_tbl_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_tbl_tests.log | head -20; tail -3 gpurun_out/${TAG}_tbl_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tbl_tests.log
timeout -k 10 120 python tools/diag_table.py > gpurun_out/${TAG}_diag_table.log 2>&1; tail -2 gpurun_out/${TAG}_diag_table.log
timeout -k 10 120 python tools/diag_dec.py > gpurun_out/${TAG}_diag_dec.log 2>&1; head -3 gpurun_out/${TAG}_diag_dec.log
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/${TAG}_gpu_tests.log | head; tail -3 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | python tools/bench_brief.py
for st in hist encode; do timeout -k 10 120 python tools/abl_time.py --stage $st; done
