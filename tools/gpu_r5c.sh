# Round-5 call c: table kernels vs the oracle on large counts (C4 failure), table phases,
# pack A/B (next-block prefetch before the stores vs after; no-store ablation), all GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r5c}
mkdir -p gpurun_out
timeout -k 10 200 python tools/dbg_table.py > gpurun_out/${TAG}_dbg_table.log 2>&1; cat gpurun_out/${TAG}_dbg_table.log | grep -v amdgpu.ids
timeout -k 10 120 python tools/diag_table.py > gpurun_out/${TAG}_diag_table.log 2>&1; tail -1 gpurun_out/${TAG}_diag_table.log
L=gpurun_out/${TAG}_abl.log
: > $L
for r in 1 2; do
  timeout -k 10 120 python tools/abl_time.py --stage encode --opt pack_prefetch=2 >> $L 2>&1 || { tail -3 $L; exit 1; }
  timeout -k 10 120 python tools/abl_time.py --stage encode --opt pack_prefetch=1 >> $L 2>&1 || { tail -3 $L; exit 1; }
done
for lib in _abl_p_nostore _abl_p_none; do
  DC_CORE_LIB=$PWD/tools/$lib/libdc_core.so timeout -k 10 120 python tools/abl_time.py --stage encode --opt pack_prefetch=2 >> $L 2>&1 || { tail -3 $L; exit 1; }
  DC_CORE_LIB=$PWD/tools/$lib/libdc_core.so timeout -k 10 120 python tools/abl_time.py --stage encode --opt pack_prefetch=1 >> $L 2>&1 || { tail -3 $L; exit 1; }
done
grep '^{' $L
timeout -k 10 500 python -u -m pytest tests/ -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_gpu_tests.log | head; tail -1 gpurun_out/${TAG}_gpu_tests.log
