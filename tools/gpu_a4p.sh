#!/bin/bash
# conv_gemm_a4 as a tile walk (VP3D_A4_WALK=2 -- VP3D_A4_PERSIST=1 when r03w ran: one workgroup per CU, the next tile's first
# two K-tiles staged before the epilogue stores) vs one tile per workgroup: bit identity vs q64
# and the oracle in both forms (pytest; config 4 at B = 65,536 too), harness time on the
# block-1 shapes, the bench.
# Usage: bash tools/gpu_a4p.sh TAG   (outputs under gpurun_out/TAG)
set -o pipefail
TAG=${1:-a4p}
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
T="python -u -m pytest tests/test_gpu_lifter.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k"
run pytest_a4 300 $T "a4 or config4"
VP3D_A4_WALK=2 run pytest_a4p 300 $T "a4 or config4"
G=tools/ubench/gemm_check
M=221184
for r in 1 2; do
  run gc_a4_k3_$r 120 $G a4 $M 1024 1024 1 3 0
  VP3D_A4_WALK=2 run gc_a4p_k3_$r 120 $G a4 $M 1024 1024 1 3 0
  run gc_a4_1x1_$r 120 $G a4 $M 1024 1024 1 1 1
  VP3D_A4_WALK=2 run gc_a4p_1x1_$r 120 $G a4 $M 1024 1024 1 1 1
done
B="python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --parity-windows 4 --no-extras"
for r in 1 2; do
  run bench_a4_$r 300 $B
  VP3D_A4_WALK=2 run bench_a4p_$r 300 $B
done
for f in bench_a4_1 bench_a4p_1 bench_a4_2 bench_a4p_2; do
  echo "$f: $(python tools/bench_brief.py $OUT/$f.log)"
done
