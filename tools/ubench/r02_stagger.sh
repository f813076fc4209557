#!/bin/bash
# q64 epilogue staggering: first-round workgroups of CU group g sleep g * iters x ~4 us, so
# the chip's tile epilogues (output + residual bursts) stop coinciding.  Block-1 1x1 (+
# residual) and k3 shapes at B = 8192 (M = 221184).  VP3D_STAGGER=iters,groups.
set -o pipefail
cd "$(dirname "$0")"
M=${M:-221184}
for st in ${STAGGERS:-0,1 1,2 2,2 3,2 1,4 2,4 1,8}; do
  for shape in "1024 1024 1 1 1" "1024 1024 1 3 0"; do
    echo -n "stagger $st shape $shape: "
    VP3D_STAGGER=$st timeout -k 5 120 ./gemm_check q64 $M $shape > /tmp/gc.log 2>&1 || { echo "rc=$?"; tail -3 /tmp/gc.log; exit 1; }
    tail -1 /tmp/gc.log
  done
done
