#!/bin/bash
# A/B of the one-wave-per-SIMD AGPR GEMM (conv_gemm_a4.hip, VP3D_GEMM=a4) against q64:
# bit identity through the library, harness parity + time on the block-1 shapes
# (random bf16, alternating kernels in separate processes; a4g = a4 with global_load_lds
# instead of buffer-resource DMA), and the bench's per-layer
# times at B = 65,536 under each kernel.
# Usage: bash tools/gpu_a4.sh TAG   (outputs under gpurun_out/TAG)
set -o pipefail
TAG=${1:-a4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(tail -1 $OUT/$name.log | cut -c1-250)"
  if [ $rc -ne 0 ]; then tail -15 $OUT/$name.log; exit $rc; fi
}
run pytest_a4 300 python -u -m pytest tests/test_gpu_lifter.py -k "a4 or override" -x -v -p no:cacheprovider --timeout 240 --timeout-method thread
G=tools/ubench/gemm_check
M=221184
for r in 1 2; do
  for k in q64 a4; do
    run gc_${k}_k3_$r 120 $G $k $M 1024 1024 1 3 0
    run gc_${k}_1x1_$r 120 $G $k $M 1024 1024 1 1 1
  done
  VP3D_A4_DMA=global run gc_a4g_k3_$r 120 $G a4 $M 1024 1024 1 3 0
done
B="python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --parity-windows 4 --no-extras"
run bench_q64 300 $B
VP3D_GEMM=a4 run bench_a4 300 $B
run bench_q64b 300 $B
VP3D_GEMM=a4 run bench_a4b 300 $B
for f in bench_q64 bench_a4 bench_q64b bench_a4b; do
  echo "$f: $(python tools/bench_brief.py $OUT/$f.log)"
done
