# (switch in the working tree at the time, not committed) Fused C5 histogram with two blocks in flight (hist_prefetch=2) against one (=1), same process
# order interleaved: the C5 encode's kernels
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r5fh_fe_hist_pf_ab.log
: > $O
for r in 1 2 3; do
  for v in 1 2; do
    timeout -k 10 150 python tools/abl_time.py --stage c5_enc --cfg C5 --nary 16 --iters 10 --warm 10 --opt hist_prefetch=$v --tag pf$v >> $O 2>&1 || { tail -3 $O; exit 1; }
  done
done
grep '^{' $O | cut -c1-300
