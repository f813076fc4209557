#!/bin/bash
# PMC passes over one gemm_check run (tool). Usage: bash tools/ubench/pmc_gemm.sh TAG "gemm_check args" "CTRS1" ["CTRS2" ...]
set -o pipefail
TAG=$1; shift; ARGS=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc$i -o run -- tools/ubench/gemm_check $ARGS > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pass $i [$C] rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $OUT/pmc$i.log; exit $rc; fi
done
