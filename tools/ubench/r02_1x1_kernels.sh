#!/bin/bash
# 1x1 + residual layers on q64 vs 8p (8p takes outputs below 2^31 bytes only): block-2 (M = 589,824) at
# B = 65,536 and block-1 at B = 8,192 (M = 221,184), alternating twice.
set -o pipefail
cd "$(dirname "$0")"
for rep in 1 2; do
for k in q64 8p; do
  for m in ${MS:-589824 221184}; do
    echo -n "$k M=$m 1x1+res: "
    timeout -k 5 100 ./gemm_check $k $m 1024 1024 1 1 1 > /tmp/gc.log 2>&1; rc=$?
    grep -o "bad=[0-9]*" /tmp/gc.log | tr '\n' ' '; tail -1 /tmp/gc.log
    if [ $rc -ne 0 ]; then echo "rc=$rc"; exit $rc; fi
  done
done
done
