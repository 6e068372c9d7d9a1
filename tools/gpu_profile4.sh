# Round-4 profiling call (run under gpurun): GPU tests, bench line (with CPU baseline),
# rocprofv3 --stats of the same command (+ JSON summary for bench.py), PMC passes (+ traffic
# JSON), configs C3-C5, nybble bench lines (static, adaptive) with their rocprof stats.
# usage: bash tools/gpu_profile3.sh TAG [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r4x}
mkdir -p gpurun_out
if [ -z "$2" ]; then
  timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/${TAG}_gpu_tests.log | head; tail -3 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_gpu_tests.log
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --no-cpu > gpurun_out/${TAG}_rocprof_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_rocprof_bench.log; exit 1; }
ST=$(ls gpurun_out/${TAG}_prof/*/run_kernel_stats.csv gpurun_out/${TAG}_prof/run_kernel_stats.csv 2>/dev/null | head -1)
cp $ST gpurun_out/${TAG}_kernel_stats.csv && python tools/rocprof_report.py gpurun_out/${TAG}_kernel_stats.csv gpurun_out/${TAG}_rocprof.json > /dev/null || exit 1
mkdir -p profiles && cp gpurun_out/${TAG}_rocprof.json profiles/   # (on the box: bench.py reads it next)
bash tools/pmc.sh gpurun_out/${TAG}_pmc || exit 1
python tools/pmc_report.py gpurun_out/${TAG}_pmc gpurun_out/${TAG}_pmc_traffic.json > gpurun_out/${TAG}_pmc.txt && cp gpurun_out/${TAG}_pmc_traffic.json profiles/
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'frac', r['frac'], r['frac_rocprof'], r['frac_vs_copy'], 'enc', r['encode_frac'], 'dec', r['decode_frac'], 'copy', r['copy_probe_GBps'], 'ok', d['roundtrip_ok'], 'cpu', d.get('cpu_baseline', {}).get('value'))"
bash tools/cfg_bench.sh || exit 1
for m in static adaptive; do
  timeout -k 10 400 python bench.py --codec nybble --mode $m > gpurun_out/${TAG}_nyb_$m.log 2>&1 || { tail -5 gpurun_out/${TAG}_nyb_$m.log; exit 1; }
  tail -1 gpurun_out/${TAG}_nyb_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('nyb $m', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('encode_frac'), r.get('decode_frac'), d.get('decode_sample'), d.get('cpu_baseline', {}).get('value'), d['roundtrip_ok'])"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_nprof_$m -o run --output-format csv -- python bench.py --codec nybble --mode $m --no-cpu > gpurun_out/${TAG}_nyb_${m}_rocprof.log 2>&1 || { tail -5 gpurun_out/${TAG}_nyb_${m}_rocprof.log; exit 1; }
  ST=$(ls gpurun_out/${TAG}_nprof_$m/*/run_kernel_stats.csv gpurun_out/${TAG}_nprof_$m/run_kernel_stats.csv 2>/dev/null | head -1)
  cp $ST gpurun_out/${TAG}_nyb_${m}_kernel_stats.csv
done
# the fused C5 line beside the two stages (same box), and the nybble PMC traffic
timeout -k 10 300 python bench.py --no-cpu --frontend --cfg C5 --nary 16 --two-stage > gpurun_out/${TAG}_C5_two.log 2>&1 || { tail -5 gpurun_out/${TAG}_C5_two.log; exit 1; }
tail -1 gpurun_out/${TAG}_C5_two.log | python tools/bench_brief.py
bash tools/gpu_nyb_pmc.sh ${TAG} > /dev/null || exit 1
echo profile4 done
