# One profiling call (run under gpurun): GPU parity tests, bench (with CPU baseline),
# rocprofv3 kernel stats of the bench, PMC passes. Usage: bash tools/gpu_profile.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-rX}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -20 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --no-cpu > gpurun_out/${TAG}_rocprof_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_rocprof_bench.log; exit 1; }
bash tools/pmc.sh gpurun_out/${TAG}_pmc || exit 1
python tools/pmc_report.py gpurun_out/${TAG}_pmc gpurun_out/${TAG}_pmc_traffic.json > gpurun_out/${TAG}_pmc.txt
cat gpurun_out/${TAG}_pmc.txt | head -80
