#!/bin/bash
# conv_gemm_a4 schedule variants and ablations (VP3D_A4_V: 1 no loop DMA, 2 no loop
# fragment reads, 3 neither -- wrong results, timing only; 4 DMA front-loaded, 8 memory
# instructions spread between MFMAs, 12 both) on the block-1 shapes (random bf16,
# tools/ubench/gemm_check), PMC MFMA-busy / issue-wait / clock of a4 vs q64, and the bench
# under a4 variants.
# Usage: bash tools/gpu_a4v.sh TAG   (outputs under gpurun_out/TAG)
set -o pipefail
TAG=${1:-a4v}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(tail -1 $OUT/$name.log | cut -c1-200)"
  # the ablations compute wrong results on purpose: gemm_check exits 1 on a mismatch
  if [ $rc -gt 1 ]; then tail -15 $OUT/$name.log; exit $rc; fi
}
G=tools/ubench/gemm_check
M=221184
for r in 1 2; do
  run gc_q64_k3_$r 120 $G q64 $M 1024 1024 1 3 0
  for v in 0 1 2 3 4 8 12; do
    VP3D_A4_V=$v run gc_a4v${v}_k3_$r 120 $G a4 $M 1024 1024 1 3 0
  done
  for v in 0 8 12; do
    VP3D_A4_V=$v run gc_a4v${v}_1x1_$r 120 $G a4 $M 1024 1024 1 1 1
  done
done
P="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
run pmc_q64 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_q64 -o run -- $G q64 $M 1024 1024 1 3 0
VP3D_A4_V=0 run pmc_a4 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_a4 -o run -- $G a4 $M 1024 1024 1 3 0
VP3D_A4_V=8 run pmc_a4v8 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_a4v8 -o run -- $G a4 $M 1024 1024 1 3 0
B="python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --parity-windows 4 --no-extras"
for v in 0 8 12; do
  VP3D_GEMM=a4 VP3D_A4_V=$v run bench_a4v$v 300 $B
done
for v in 0 8 12; do
  echo "bench_a4v$v: $(python tools/bench_brief.py $OUT/bench_a4v$v.log)"
done
