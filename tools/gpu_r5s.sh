# Round-5 call s: per-lane nybble kernels with 128-B output lines: tests, A/B against the last
# commit's library, FETCH/WRITE of the batch decode and the DCNK encode alone (abl_time stages).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r5s}
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread -k "nyb or nybble or chunked or batch" > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
bash tools/gpu_ab_old.sh ${TAG} "batch C1 2" "chunk_enc C1 2" || exit 1
for st in batch chunk_enc; do
  D=gpurun_out/${TAG}_pmc_$st; rm -rf $D; mkdir -p $D; i=0
  for PASS in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $PASS -d $D/p$i -o run --output-format csv -- python tools/abl_time.py --stage $st --cfg C1 --iters 2 --warm 1 > $D/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $D/p$i.log; exit 1; }
  done
  PMC_ALL=1 python tools/pmc_report.py $D gpurun_out/${TAG}_${st}_traffic.json C1-$st 268435456 0 > gpurun_out/${TAG}_${st}_pmc.txt || exit 1
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_${st}_traffic.json'))['kernels']; print('$st', {k: (round(v['read_bytes']/1e9,3), round(v['write_bytes']/1e9,3)) for k, v in d.items() if 'nyb' in k})"
done
