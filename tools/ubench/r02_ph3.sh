#!/bin/bash
# q64 with Q2 + Q3 merged into one 32-MFMA phase (VP3D_ABL=4: 6 barriers per K-tile instead
# of 8) vs default; block-1 shapes at B = 65,536, alternating twice.
set -o pipefail
cd "$(dirname "$0")"
for rep in 1 2; do
for a in 0 4; do
  for shape in "1769472 1024 1024 1 3 0" "1769472 1024 1024 1 1 1"; do
    echo -n "abl $a shape $shape: "
    VP3D_ABL=$a timeout -k 5 100 ./gemm_check q64 $shape > /tmp/gc.log 2>&1; rc=$?
    grep "max|d|" /tmp/gc.log | cut -c1-120 | tr '\n' ' '; tail -1 /tmp/gc.log
    if [ $rc -ne 0 ]; then echo "rc=$rc"; exit $rc; fi
  done
done
done
