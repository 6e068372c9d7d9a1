# PMC of the decode kernels per variant (run under gpurun): bash tools/gpu_pmc_dec.sh "0 1"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcdec
for V in ${1:-0 1}; do
  i=0
  for PASS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
              "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $PASS -d gpurun_out/pmcdec/v${V}/p$i -o run --output-format csv -- python tools/kern_ab.py --stage decode --option decode_variant --values $V --rounds 1 --iters 2 > gpurun_out/pmcdec/v${V}_p$i.log 2>&1
    rc=$?
    echo "variant $V pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmcdec/v${V}_p$i.log; exit $rc; fi
  done
done
for V in ${1:-0 1}; do echo "== variant $V"; python tools/pmc_report.py gpurun_out/pmcdec/v$V; done > gpurun_out/pmcdec/report.txt 2>&1 || true
