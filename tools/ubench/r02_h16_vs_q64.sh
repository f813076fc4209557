#!/bin/bash
# 128x128 register-staged kernel (2 workgroups per CU by LDS) vs q64 on the block-1 shapes at
# B = 65,536 (M = 1,769,472): 1x1 + residual, 1x1, k3.
set -o pipefail
cd "$(dirname "$0")"
M=${M:-1769472}
for k in q64 h16; do
  for shape in "1024 1024 1 1 1" "1024 1024 1 1 0" "1024 1024 1 3 0"; do
    echo -n "$k shape $shape: "
    VP3D_GEMM=$k timeout -k 5 120 ./gemm_check h16 $M $shape > /tmp/gc.log 2>&1 || { echo "rc=$?"; tail -3 /tmp/gc.log; exit 1; }
    tail -1 /tmp/gc.log
  done
done
