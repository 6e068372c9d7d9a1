# where the HIP-event split loses time with lanes in flight (tools/bench_split_diag.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for f in 2 1; do
  timeout -k 10 240 python tools/bench_split_diag.py --no-cpu --in-flight $f > gpurun_out/r5w_diag_f$f.log 2>&1 || { tail -5 gpurun_out/r5w_diag_f$f.log; exit 1; }
  echo "== in-flight $f"; grep diag gpurun_out/r5w_diag_f$f.log
  tail -1 gpurun_out/r5w_diag_f$f.log | python tools/bench_brief.py
done
