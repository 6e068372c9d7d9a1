# copy-probe shape (bench line's reference rate) + the read-only rate beside it
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r3r_bench.log 2>&1 || { tail -5 gpurun_out/r3r_bench.log; exit 1; }
tail -1 gpurun_out/r3r_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], 'copy', r['copy_probe_GBps'], 'frac_vs_copy', r['frac_vs_copy'], 'dec', r['decode_frac'], r['decode_frac_vs_copy'], 'enc', r['encode_frac'], r['encode_frac_vs_copy'], {k:v['ms'] for k,v in d['kernels'].items()})"
timeout -k 10 60 tools/ubench/_gap2 > /dev/null
