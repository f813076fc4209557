#!/bin/bash
# q64 epilogue split on the 1x1 shapes at B = 65,536 (M = 1,769,472): full kernel (0), output
# stores dropped (1), no epilogue (2), epilogue without the residual loads (3).
set -o pipefail
cd "$(dirname "$0")"
M=${M:-1769472}
for a in 0 1 2 3; do
  for shape in "1024 1024 1 1 1" "1024 1024 1 1 0"; do
    echo -n "abl $a shape $shape: "
    VP3D_ABL=$a timeout -k 5 120 ./gemm_check q64 $M $shape > /tmp/gc.log 2>&1; rc=$?; tail -1 /tmp/gc.log
    if [ $rc -gt 1 ]; then echo "rc=$rc"; exit $rc; fi
  done
done
