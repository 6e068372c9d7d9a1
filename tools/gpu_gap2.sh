set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/gap2 -o run --output-format csv -- tools/ubench/_gap2 > gpurun_out/gap2.log 2>&1 || { tail -5 gpurun_out/gap2.log; exit 1; }
F=$(ls gpurun_out/gap2/*/run_kernel_trace.csv gpurun_out/gap2/run_kernel_trace.csv 2>/dev/null | head -1)
python - "$F" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
prev = None; stats = {}
for r in rows:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp']); name = r['Kernel_Name'].split('(')[0]
    if prev is not None:
        key = prev[0] + ' -> ' + name
        stats.setdefault(key, []).append((s - prev[1]) / 1000)
    stats.setdefault('dur ' + name, []).append((e - s) / 1000)
    prev = (name, e)
for k, v in stats.items():
    v = sorted(v); print(f"{k:60s} n={len(v):3d} median {v[len(v)//2]:8.2f} us  min {v[0]:8.2f}")
PY
