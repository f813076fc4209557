#!/bin/bash
# conv_gemm_a4 per-workgroup stamps (tools/ubench/gemm_check a4t: prologue / K loop /
# epilogue split, cycles in the mid waits) and epilogue ablations (VP3D_ABL 8: stores
# dropped, 16: no epilogue; +4: stamped) on the block-1 shapes, random bf16.
# Usage: bash tools/gpu_a4t.sh TAG   (outputs under gpurun_out/TAG)
set -o pipefail
TAG=${1:-a4t}
OUT=gpurun_out/$TAG
mkdir -p $OUT
G=tools/ubench/gemm_check
M=221184
for sh in "3 0" "1 1"; do
  n=$(echo $sh | tr ' ' _)
  for a in 4 12 20; do
    VP3D_ABL=$a timeout -k 10 120 $G a4t $M 1024 1024 1 $sh > $OUT/a4t_${n}_$a.log 2>&1
    rc=$?; [ $rc -gt 1 ] && exit $rc
    echo "$n ABL=$a: $(grep 'trace' $OUT/a4t_${n}_$a.log | head -2 | tr '\n' ' ')"
  done
  for a in 0 8 16; do
    VP3D_ABL=$a timeout -k 10 120 $G a4 $M 1024 1024 1 $sh > $OUT/a4_${n}_$a.log 2>&1
    rc=$?; [ $rc -gt 1 ] && exit $rc
    echo "$n ABL=$a: $(tail -1 $OUT/a4_${n}_$a.log)"
  done
done
