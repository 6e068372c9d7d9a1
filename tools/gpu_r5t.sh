# Steps in flight (tools/inflight_probe.py): C2 and fused C5, one context against two on two streams
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python tools/inflight_probe.py C2 2 > gpurun_out/r5t_inflight_C2.log 2>&1 || { tail -5 gpurun_out/r5t_inflight_C2.log; exit 1; }
cat gpurun_out/r5t_inflight_C2.log
timeout -k 10 240 python tools/inflight_probe.py C5 16 --frontend > gpurun_out/r5t_inflight_C5.log 2>&1 || { tail -5 gpurun_out/r5t_inflight_C5.log; exit 1; }
cat gpurun_out/r5t_inflight_C5.log
