# (A/B kernel in the working tree at the time, not committed; profiles/r5h32_hist_cols_ab.log) the histogram with 32 lane columns at 3 workgroups
# per CU (hist_prefetch 4 / 5 = 1 / 2 blocks in flight) against the default (2): the histogram
# against torch.bincount, the encode+decode step round trip, on 1 GiB and on a ragged size
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r5h32_hist_cols_ab.log
: > $O
timeout -k 10 200 python tools/kern_ab.py --stage step --option hist_prefetch --values 2,5 --size 1000003 --rounds 2 >> $O 2>&1 || { tail -5 $O; exit 1; }
timeout -k 10 200 python tools/kern_ab.py --stage hist --option hist_prefetch --values 2,4,5 --size 70001 --rounds 2 >> $O 2>&1 || { tail -5 $O; exit 1; }
timeout -k 10 200 python tools/kern_ab.py --stage hist --option hist_prefetch --values 2,4,5 >> $O 2>&1 || { tail -5 $O; exit 1; }
timeout -k 10 200 python tools/kern_ab.py --stage step --option hist_prefetch --values 2,5,4 >> $O 2>&1 || { tail -5 $O; exit 1; }
timeout -k 10 200 python tools/kern_ab.py --stage hist --option hist_prefetch --values 2,4,5 --cfg C4 >> $O 2>&1 || { tail -5 $O; exit 1; }
grep -v amdgpu.ids $O
