# Round-5 call n: MTF walk with a round's 8 granules loaded together: nybble GPU tests, same-box
# A/B of the adaptive encode against the previous library (tools/_old), and FETCH/WRITE passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r5n}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread -k "nyb or nybble or mtf or adaptive" > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_tests.log | head -20; tail -3 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
L=gpurun_out/${TAG}_abl.log
: > $L
for r in 1 2; do
  timeout -k 10 120 python tools/abl_time.py --stage nyb_adaptive --cfg C1 --iters 10 --warm 5 >> $L 2>&1 || { tail -3 $L; exit 1; }
  DC_CORE_LIB=tools/_old/libdc_core.so timeout -k 10 120 python tools/abl_time.py --stage nyb_adaptive --cfg C1 --iters 10 --warm 5 >> $L 2>&1 || { tail -3 $L; exit 1; }
done
grep '^{' $L
O=gpurun_out/${TAG}_pmc
rm -rf $O; mkdir -p $O
i=0
for PASS in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $PASS -d $O/p$i -o run --output-format csv -- python tools/abl_time.py --stage nyb_adaptive --cfg C1 --iters 2 --warm 1 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
PMC_ALL=1 PMC_KEEP_TEMPLATE=1 python tools/pmc_report.py $O gpurun_out/${TAG}_nyb_adaptive_pmc_traffic.json C1-nyb-adaptive 1073741824 0 > gpurun_out/${TAG}_nyb_adaptive_pmc.txt || exit 1
grep -A3 "k_mtf_walk" gpurun_out/${TAG}_nyb_adaptive_pmc.txt
python -c "import json; d=json.load(open('gpurun_out/${TAG}_nyb_adaptive_pmc_traffic.json'))['kernels']; print({k: v for k, v in d.items() if 'walk' in k or 'fsm_write' in k})"
