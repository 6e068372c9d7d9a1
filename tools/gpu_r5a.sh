# Round-5 first call (run under gpurun): GPU tests, the bench line, and the per-kernel
# ablations of the three C2 kernels (decode, histogram, pack) against the in-tree library.
# usage: bash tools/gpu_r5a.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r5a}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/${TAG}_gpu_tests.log | head; tail -3 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | python tools/bench_brief.py
L=gpurun_out/${TAG}_abl.log
: > $L
for st in decode hist encode; do
  timeout -k 10 120 python tools/abl_time.py --stage $st >> $L 2>&1 || { tail -3 $L; exit 1; }
done
for lib in _abl_synth _abl_lut _abl_nodec _abl_nost _abl_nodec_nost; do
  DC_CORE_LIB=$PWD/tools/$lib/libdc_core.so timeout -k 10 120 python tools/abl_time.py --stage decode >> $L 2>&1 || { tail -3 $L; exit 1; }
done
for lib in _abl_h_noatom _abl_h_nored _abl_h_none; do
  DC_CORE_LIB=$PWD/tools/$lib/libdc_core.so timeout -k 10 120 python tools/abl_time.py --stage hist >> $L 2>&1 || { tail -3 $L; exit 1; }
done
for lib in _abl_p_nolut _abl_p_noor _abl_p_none; do
  DC_CORE_LIB=$PWD/tools/$lib/libdc_core.so timeout -k 10 120 python tools/abl_time.py --stage encode >> $L 2>&1 || { tail -3 $L; exit 1; }
done
for st in decode hist encode; do
  timeout -k 10 120 python tools/abl_time.py --stage $st --tag base_again >> $L 2>&1 || { tail -3 $L; exit 1; }
done
grep '^{' $L
echo r5a done
