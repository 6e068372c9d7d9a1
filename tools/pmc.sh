#!/bin/bash
# PMC passes over a short bench run (one counter group per pass; no --sys-trace/--pmc mixing).
# usage: tools/pmc.sh OUTDIR [bench args...]
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}; shift
ARGS=${@:---no-cpu --steps 2 --warmup 1 --profile-steps 1}
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for PASS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
            "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $PASS -d $OUT/p$i -o run --output-format csv -- python bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($PASS) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
