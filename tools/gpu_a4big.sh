#!/bin/bash
# conv_gemm_a4 per-workgroup stamps at the B = 65,536 block-1 shapes (tools/ubench/gemm_check
# a4t, no reference check), and the q64 / a4 times there.
set -o pipefail
TAG=${1:-a4big}
OUT=gpurun_out/$TAG
mkdir -p $OUT
G=tools/ubench/gemm_check
M=1769472
export VP3D_NOCHECK=1
for sh in "3 0" "1 1"; do
  n=$(echo $sh | tr ' ' _)
  timeout -k 10 120 $G a4t $M 1024 1024 1 $sh > $OUT/a4t_$n.log 2>&1 || exit $?
  echo "$n: $(grep 'trace: \(wave\|kernel\)' $OUT/a4t_$n.log | tr '\n' ' ')"
  for k in a4 q64; do
    timeout -k 10 120 $G $k $M 1024 1024 1 $sh > $OUT/${k}_$n.log 2>&1 || exit $?
    echo "$n $k: $(tail -1 $OUT/${k}_$n.log)"
  done
done
