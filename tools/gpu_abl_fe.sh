set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/fe_time.py 10 > gpurun_out/abl_base.log 2>&1 && tail -1 gpurun_out/abl_base.log && \
DC_CORE_LIB=$GRAFT_REPO_ROOT/tools/_diag_nt/libdc_core.so timeout -k 10 300 python tools/fe_time.py 10 > gpurun_out/abl_nt.log 2>&1 && tail -1 gpurun_out/abl_nt.log
