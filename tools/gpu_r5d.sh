# Round-5 call d: pack structure ablations (loads / stores / LDS work removed one by one).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r5d}
mkdir -p gpurun_out
L=gpurun_out/${TAG}_abl.log
: > $L
timeout -k 10 120 python tools/abl_time.py --stage encode >> $L 2>&1 || { tail -3 $L; exit 1; }
for lib in _abl_p_noload _abl_p_nostore _abl_p_nolst _abl_p_memonly _abl_p_skel _abl_p_none; do
  DC_CORE_LIB=$PWD/tools/$lib/libdc_core.so timeout -k 10 120 python tools/abl_time.py --stage encode >> $L 2>&1 || { tail -3 $L; exit 1; }
done
timeout -k 10 120 python tools/abl_time.py --stage encode --tag base_again >> $L 2>&1 || { tail -3 $L; exit 1; }
grep '^{' $L
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -q --timeout 200 --timeout-method thread -k "c4" > gpurun_out/${TAG}_c4.log 2>&1; tail -1 gpurun_out/${TAG}_c4.log
