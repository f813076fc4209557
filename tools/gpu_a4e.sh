#!/bin/bash
# conv_gemm_a4 after an epilogue change: bit identity vs q64 and the oracle (pytest), harness
# time and stamps on the block-1 shapes, the bench (a4 default) vs VP3D_GEMM=q64.
# Usage: bash tools/gpu_a4e.sh TAG   (outputs under gpurun_out/TAG)
set -o pipefail
TAG=${1:-a4e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(tail -1 $OUT/$name.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then tail -15 $OUT/$name.log; exit $rc; fi
}
run pytest_a4 400 python -u -m pytest tests/test_gpu_lifter.py tests/test_gpu_golden.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
G=tools/ubench/gemm_check
M=221184
for r in 1 2; do
  for k in q64 a4; do
    run gc_${k}_k3_$r 120 $G $k $M 1024 1024 1 3 0
    run gc_${k}_1x1_$r 120 $G $k $M 1024 1024 1 1 1
  done
done
run a4t_k3 120 $G a4t $M 1024 1024 1 3 0
run a4t_1x1 120 $G a4t $M 1024 1024 1 1 1
grep trace $OUT/a4t_k3.log | head -2; grep trace $OUT/a4t_1x1.log | head -2
B="python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --parity-windows 4 --no-extras"
for r in 1 2; do
  run bench_a4_$r 300 $B
  VP3D_GEMM=q64 run bench_q64_$r 300 $B
done
for f in bench_a4_1 bench_q64_1 bench_a4_2 bench_q64_2; do
  echo "$f: $(python tools/bench_brief.py $OUT/$f.log)"
done
