#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/x3_depth.py --B 512 > gpurun_out/r04b_x3_depth.txt 2>&1
rc=$?
cat gpurun_out/r04b_x3_depth.txt
exit $rc
