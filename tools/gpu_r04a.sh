#!/bin/bash
# Round 4, step a: MFMA accumulation numerics (probes + sign-correlated bias of the split-fp16
# chains and candidate fixes) and the f16x3 shrink on the dolly windows.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 tools/ubench/mfma_rounding > gpurun_out/r04a_mfma_rounding.txt 2>&1 &&
for d in 0 1 2; do timeout -k 10 120 tools/ubench/mfma_bias 3072 512 $d; done > gpurun_out/r04a_mfma_bias.txt 2>&1 &&
timeout -k 10 120 tools/ubench/mfma_bias 1024 512 1 >> gpurun_out/r04a_mfma_bias.txt 2>&1 &&
timeout -k 10 300 python -u tools/x3_shrink.py --B 256 > gpurun_out/r04a_x3_shrink.txt 2>&1 &&
timeout -k 10 300 python -u tools/x3_shrink.py --B 256 --config4 >> gpurun_out/r04a_x3_shrink.txt 2>&1
rc=$?
cat gpurun_out/r04a_mfma_rounding.txt gpurun_out/r04a_mfma_bias.txt gpurun_out/r04a_x3_shrink.txt
exit $rc
