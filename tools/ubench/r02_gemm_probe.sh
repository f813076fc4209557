#!/bin/bash
# Round-2 GEMM probe: per-workgroup timeline of the 8p kernel (prologue / K loop /
# epilogue) on the block-1 shapes, the K sweep of the 1x1 shape, and hipBLASLt.
set -o pipefail
cd "$(dirname "$0")"
G="timeout -k 5 60 ./gemm_check"
M=221184
$G 8pt $M 1024 1024 1 1 1 | grep trace || exit $?
$G 8pt $M 1024 1024 1 3 0 | grep trace || exit $?
for cin in 512 1024 2048 3072; do $G 8p $M 1024 $cin 1 1 0 | tail -1 || exit $?; done
$G 8p $M 1024 1024 1 1 1 | tail -1 || exit $?
$G 8p $M 1024 1024 1 3 0 | tail -1 || exit $?
timeout -k 5 120 python torch_gemm.py || exit $?
