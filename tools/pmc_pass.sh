#!/bin/bash
# rocprofv3 PMC passes over a short bench run (counters only: no sys/runtime trace).
# Usage: bash tools/pmc_pass.sh TAG "CTR1 CTR2 ..." ["CTR..."] ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc$i -o run -- python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --parity-windows 4 ${BENCH_ARGS} > $OUT/pmc$i.log 2>&1
  rc=$?
  echo "pass $i [$C] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/pmc$i.log; exit $rc; fi
done
