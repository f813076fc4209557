#!/bin/bash
# Round 4 step j: sign-balanced split-fp16 weights -- output scale per depth (balanced vs not),
# the dolly / config-4 shrink diagnostic, and the config-3 / golden parity tests.
set -o pipefail
mkdir -p gpurun_out/r04j
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r04j/numerics.txt
timeout -k 10 400 python -u tools/x3_depth.py --B 512 --dtypes fp32,f16x3 --variants default,nosign > $o 2>&1 &&
timeout -k 10 300 python -u tools/x3_shrink.py --B 256 >> $o 2>&1 &&
timeout -k 10 300 python -u tools/x3_shrink.py --B 256 --config4 >> $o 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_traj.py tests/test_gpu_golden.py tests/test_gpu_lifter.py -m gpu > gpurun_out/r04j/pytest.txt 2>&1
rc=$?
cat $o; grep -E "dolly|passed|failed|Error" gpurun_out/r04j/pytest.txt | tail -15
exit $rc
