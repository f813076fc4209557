#!/bin/bash
# Round 4 step e: conversion rounding; the split-fp16 scale per depth with the q64 GEMM and the
# pack-form expand.
set -o pipefail
mkdir -p gpurun_out
o=gpurun_out/r04e.txt
timeout -k 10 60 tools/ubench/cvt_rounding > $o 2>&1 &&
echo "== VP3D_GEMM=q64" >> $o && VP3D_GEMM=q64 timeout -k 10 300 python -u tools/x3_depth.py --B 512 --dtypes fp32,f16x3 >> $o 2>&1 &&
echo "== VP3D_X3_EXPAND=pack" >> $o && VP3D_X3_EXPAND=pack timeout -k 10 300 python -u tools/x3_depth.py --B 512 --dtypes fp32,f16x3 >> $o 2>&1
rc=$?
cat $o
exit $rc
