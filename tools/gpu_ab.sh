# run tools/kern_ab.py under gpurun: bash tools/gpu_ab.sh TAG kern_ab args...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 300 python tools/kern_ab.py "$@" > gpurun_out/ab_${TAG}.log 2>&1
rc=$?
tail -8 gpurun_out/ab_${TAG}.log
exit $rc
