#!/bin/bash
# PMC passes over the expand-conv harness (RB = 4, stores on): wave-cycle breakdown,
# instruction mix, LDS, TA busy.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02p}; mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE"
P3="TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
i=0
for C in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  mkdir -p $OUT/pmc$i
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc$i -o run -- tools/ubench/expand_check 65536 ${RB:-4} 0 > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $OUT/pmc$i.log; exit $rc; fi
done
