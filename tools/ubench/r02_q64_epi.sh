#!/bin/bash
# q64 per-tile epilogue cost: the full kernel, stores dropped by the range check
# (VP3D_ABL=1) and no epilogue (VP3D_ABL=2), on the block-1 1x1 (+ residual) and k3 shapes.
set -o pipefail
cd "$(dirname "$0")"
M=${M:-221184}
for a in ${ABLS:-0 1 2}; do
  for shape in "1024 1024 1 1 0" "1024 1024 1 1 1" "1024 1024 1 3 0"; do
    echo -n "abl $a shape $shape: "
    VP3D_ABL=$a timeout -k 5 120 ./gemm_check q64 $M $shape > /tmp/gc.log 2>&1; rc=$?; tail -1 /tmp/gc.log; if [ $rc -gt 1 ] || { [ $a = 0 ] && [ $rc -ne 0 ]; }; then echo "rc=$rc"; exit $rc; fi  # ablations fail the check (rc 1) by design
  done
done
