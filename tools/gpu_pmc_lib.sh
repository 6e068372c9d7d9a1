# PMC of one stage's kernels per library (run under gpurun): bash tools/gpu_pmc_lib.sh STAGE "base q0"
#   base = in-tree library, X = tools/_ablX/libdc_core.so; report in gpurun_out/pmclib/report.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmclib
STAGE=${1:-decode}
for V in ${2:-base}; do
  if [ $V = base ]; then unset DC_CORE_LIB; else export DC_CORE_LIB=$PWD/tools/_abl$V/libdc_core.so; fi
  i=0
  for PASS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
              "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
              "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $PASS -d gpurun_out/pmclib/$V/p$i -o run --output-format csv -- python tools/kern_ab.py --stage $STAGE --option decode_static_pct --values 60 --rounds 1 --iters 2 > gpurun_out/pmclib/${V}_p$i.log 2>&1
    rc=$?
    echo "$V pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmclib/${V}_p$i.log; exit $rc; fi
  done
done
for V in ${2:-base}; do echo "== $V"; python tools/pmc_report.py gpurun_out/pmclib/$V; done > gpurun_out/pmclib/report.txt 2>&1
cat gpurun_out/pmclib/report.txt
