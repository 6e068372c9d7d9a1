# Option sweeps on the current kernels (same process, interleaved rounds): the decoder's static
# share and the histogram's blocks in flight
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r5sw_option_sweeps.log
: > $O
timeout -k 10 200 python tools/kern_ab.py --stage decode --option decode_static_pct --values 40,60,80,100 >> $O 2>&1 || { tail -5 $O; exit 1; }
timeout -k 10 200 python tools/kern_ab.py --stage hist --option hist_prefetch --values 1,2,3 >> $O 2>&1 || { tail -5 $O; exit 1; }
timeout -k 10 200 python tools/kern_ab.py --stage decode --option decode_static_pct --values 40,60,80 --cfg C5 --nary 16 >> $O 2>&1 || { tail -5 $O; exit 1; }
grep -v amdgpu.ids $O | tail -40
