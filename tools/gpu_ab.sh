#!/bin/bash
# GPU session for kernel A/B work: GPU tests, then bench.py once per env setting.
# Usage: bash tools/gpu_ab.sh TAG "ENV1" "ENV2" ...   (e.g. "VP3D_BIG_TILE=256")
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -s -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2
if [ $rc -gt 1 ]; then exit $rc; fi
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/bench_$i.log 2>&1 || exit $?
  echo "[$E] $(python tools/bench_brief.py $OUT/bench_$i.log)"
done
