# Steps in flight: HIP-event split on lane 0 with / without a second lane (tools/inflight_probe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python tools/inflight_probe.py C2 2 --rounds 2 > gpurun_out/r5v_inflight_C2.log 2>&1 || { tail -5 gpurun_out/r5v_inflight_C2.log; exit 1; }
cat gpurun_out/r5v_inflight_C2.log
