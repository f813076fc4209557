#!/bin/bash
# Round 4 step h: the split-fp16 output scale per depth, per GEMM / expand variant.
set -o pipefail
mkdir -p gpurun_out/r04h
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/x3_depth.py --B 512 --dtypes fp32,f16x3 --variants default,q64,pack,q64pack > gpurun_out/r04h/x3_depth.txt 2>&1
rc=$?
cat gpurun_out/r04h/x3_depth.txt
exit $rc
