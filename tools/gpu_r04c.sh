#!/bin/bash
# Round 4 step c: split-fp16 scale per depth; the serve end protocol and the trajectory-lifter
# --evaluate path on the GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/x3_depth.py --B 512 > gpurun_out/r04c_x3_depth.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stream.py tests/test_run_eval_seq.py -m gpu > gpurun_out/r04c_pytest.txt 2>&1
rc=$?
cat gpurun_out/r04c_x3_depth.txt; tail -30 gpurun_out/r04c_pytest.txt
exit $rc
