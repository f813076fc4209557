#!/bin/bash
# split-fp16 (f16x3) checks after an a4 X3 change (bit identity vs q64, the fp32-gated goldens
# and config-4 tilings), the f16x3 bench line, then the secondary-configuration refresh.
set -o pipefail
TAG=${1:-x3tail}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_lifter.py tests/test_gpu_golden.py tests/test_gpu_traj.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "x3 or a4" > $OUT/pytest_x3.log 2>&1
rc=$?; echo "pytest_x3 rc=$rc: $(tail -1 $OUT/pytest_x3.log)"; [ $rc -ne 0 ] && { tail -20 $OUT/pytest_x3.log; exit $rc; }
timeout -k 10 300 python bench.py --dtype f16x3 --steps 10 --warmup 3 --cpu-seconds 0 --no-extras > $OUT/bench_x3.log 2>&1 || { tail -5 $OUT/bench_x3.log; exit 1; }
echo "bench_x3: $(python tools/bench_brief.py $OUT/bench_x3.log)"
bash tools/gpu_tail_r03.sh $TAG
