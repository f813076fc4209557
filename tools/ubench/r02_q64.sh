#!/bin/bash
# q64 (64-deep K-tiles, whole-line DMA) vs 8p on the block-1 shapes: parity vs the naive
# reference kernel and time (random bf16 data).
set -o pipefail
cd "$(dirname "$0")"
G="timeout -k 5 60 ./gemm_check"
M=221184
for k in ${KERNS:-q64 8p}; do
  $G $k $M 1024 1024 1 1 0 | tail -2 || exit $?
  $G $k $M 1024 1024 1 1 1 | tail -2 || exit $?
  $G $k $M 1024 1024 1 3 0 | tail -2 || exit $?
  $G $k 1000 1024 1024 1 3 1 | tail -2 || exit $?
done
