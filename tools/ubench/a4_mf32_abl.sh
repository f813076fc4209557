#!/bin/bash
# bf16 a4 K loop: 16x16x32 (ABL 0) vs the 32x32x16 issue pattern (ABL 64, results wrong),
# each with and without the loop DMA (1 / 65), block-1 k3 (stride 3) and 1x1 shapes,
# interleaved rounds (tools/ubench/gemm_check built by build_gemm_check.sh)
set -o pipefail
cd "$(dirname "$0")"
M=${M:-221184}
for r in 1 2 3; do
  for abl in 0 64 1 65; do
    echo -n "round $r abl $abl k3: "
    VP3D_ABL=$abl VP3D_NOCHECK=1 VP3D_STRIDE=3 timeout -k 5 60 ./gemm_check a4 $M 1024 1024 1 3 0 | tail -1 || exit 1
    echo -n "round $r abl $abl 1x1: "
    VP3D_ABL=$abl VP3D_NOCHECK=1 timeout -k 5 60 ./gemm_check a4 $M 1024 1024 1 1 1 | tail -1 || exit 1
  done
done
