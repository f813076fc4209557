#!/bin/bash
# Main-loop efficiency probe: the same kernels on shapes where the per-tile prologue /
# epilogue is amortised (long K) and on a 4096^3-equivalent (one tile per CU).
set -o pipefail
cd "$(dirname "$0")"
G="timeout -k 5 60 ./gemm_check"
for k in ${KERNS:-q64 8p}; do
  $G $k 16384 1024 4096 1 1 0 | tail -1 || exit $?
  $G $k 16384 1024 4096 1 4 0 | tail -1 || exit $?
  $G $k 65536 1024 2048 1 8 0 | tail -1 || exit $?
done
