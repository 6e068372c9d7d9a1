# adaptive nybble line with the product library, then with a diagnostic build (same box)
# usage: bash tools/gpu_abl_mtf.sh TAG DIAG_DIR
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-abl}; D=${2:-_diag_nt2}
mkdir -p gpurun_out
brief() { python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['value'], d['roundtrip_ok'], {k: v['ms'] for k, v in d['kernels'].items()})"; }
timeout -k 10 300 python bench.py --codec nybble --mode adaptive --no-cpu > gpurun_out/${TAG}_base.log 2>&1 && tail -1 gpurun_out/${TAG}_base.log | brief base && \
DC_CORE_LIB=$GRAFT_REPO_ROOT/tools/$D/libdc_core.so timeout -k 10 300 python bench.py --codec nybble --mode adaptive --no-cpu > gpurun_out/${TAG}_diag.log 2>&1 && tail -1 gpurun_out/${TAG}_diag.log | brief diag
