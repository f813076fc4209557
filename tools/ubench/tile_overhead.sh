#!/bin/bash
# Per-tile overhead of the 256x256 conv-GEMMs: same M x N, K swept (1x1 convs with
# Cin = K, and the k3 shape), with and without a residual; M at 13.5 and 14 rounds.
set -o pipefail
cd "$(dirname "$0")"
G="timeout -k 5 60 ./gemm_check"
for k in 8p big; do
  for M in 221184 229376; do
    for cin in 1024 2048 3072; do
      $G $k $M 1024 $cin 1 1 0 | tail -1 || exit $?
    done
    $G $k $M 1024 1024 1 1 1 | tail -1 || exit $?
    $G $k $M 1024 1024 1 3 0 | tail -1 || exit $?
  done
done
