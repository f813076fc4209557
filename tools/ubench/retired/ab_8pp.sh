#!/bin/bash
# A/B of the persistent ping-pong GEMM (VP3D_GEMM=8pp) against the default dispatch:
# harness checks (1x1 + residual, k3, ragged M), GPU lifter tests under 8pp, bench lines.
set -o pipefail
OUT=gpurun_out/ab8pp; mkdir -p $OUT
cd tools/ubench
for args in "221184 1024 1024 1 1 1" "221184 1024 1024 1 3 0" "73828 1024 1024 1 1 1" "2100 1024 1024 1 3 1" "221184 1024 1024 1 1 0"; do
  for k in 8pp 8p; do timeout -k 5 60 ./gemm_check $k $args | tail -2 || exit $?; done
done > ../../$OUT/gemm.txt 2>&1
cd ../..
VP3D_GEMM=8pp timeout -k 10 300 python -u -m pytest tests/test_gpu_lifter.py tests/test_gpu_golden.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_8pp.txt 2>&1 || exit $?
i=0
for E in "VP3D_NONE=1" "VP3D_GEMM=8pp" "VP3D_NONE=1" "VP3D_GEMM=8pp"; do
  i=$((i+1))
  env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/bench_$i.log 2>&1 || exit $?
  echo "[$E] $(python tools/bench_brief.py $OUT/bench_$i.log)" | tee -a $OUT/summary.txt
done
