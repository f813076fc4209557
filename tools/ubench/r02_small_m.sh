#!/bin/bash
# Low-tile-count layers (B = 8,192 windows per GPU, i.e. config 4 at N = 8): block-4 (M = 8,192:
# 128 tiles of 256x256) and block-3 (M = 24,576: 384 tiles) k3 / 1x1 + residual on q64 vs the
# 128x128 kernel (VP3D_GEMM=h16: 4x the workgroups, two per CU), alternating twice.
set -o pipefail
cd "$(dirname "$0")"
for rep in 1 2; do
for k in q64 h16; do
  for shape in "8192 1024 1024 1 3 0" "8192 1024 1024 1 1 1" "24576 1024 1024 1 3 0" "24576 1024 1024 1 1 1"; do
    echo -n "$k shape $shape: "
    VP3D_GEMM=$k timeout -k 5 60 ./gemm_check h16 $shape > /tmp/gc.log 2>&1; rc=$?
    grep "max|d|" /tmp/gc.log | cut -c1-100 | tr '\n' ' '; tail -1 /tmp/gc.log
    if [ $rc -ne 0 ]; then echo "rc=$rc"; exit $rc; fi
  done
done
done
