#!/bin/bash
# PMC comparison of q64 vs 8p (gemm_check, block-1 k3 and 1x1+residual shapes): wave-cycle
# breakdown, MFMA busy, LDS waits / bank conflicts, TA busy, L2 hit rate.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${PMC_TAG:-r02g}; mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for k in q64 8p; do
  for shape in "221184 1024 1024 1 3 0" "221184 1024 1024 1 1 1"; do
    tag=$k-$(echo $shape | tr ' ' '_')
    mkdir -p $OUT/$tag
    i=0
    for C in "$P1" "$P2"; do
      i=$((i+1))
      timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $OUT/$tag/pmc$i -o run -- tools/ubench/gemm_check $k $shape > $OUT/$tag/pmc$i.log 2>&1
      rc=$?; echo "$tag pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $OUT/$tag/pmc$i.log; exit $rc; fi
    done
  done
done
