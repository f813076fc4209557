#!/bin/bash
# conv_gemm_a4 on the strided block-1 k3 shape at B = 65,536: one tile per workgroup (default)
# vs the tile walk (VP3D_A4_WALK=2: one workgroup per CU, the next tile's K-tiles 0 and 1
# staged in the last K-tile), interleaved runs; then the walked per-workgroup stamps.
set -o pipefail
TAG=${1:-a4walk}
OUT=gpurun_out/$TAG
mkdir -p $OUT
G=tools/ubench/gemm_check
go() {  # name, env/command...
  local name=$1; shift
  env "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(grep -E 'trace: |TFLOP|bad=' $OUT/$name.log | tr '\n' ' ' | cut -c1-300)"
  [ $rc -ne 0 ] && exit $rc
}
export VP3D_STRIDE=3 VP3D_RELU_A=1
go chk_walk VP3D_A4_WALK=2 timeout -k 10 120 $G a4 221184 1024 1024 1 3 0
for r in 1 2; do
  go k3_tile_$r VP3D_NOCHECK=1 VP3D_ITERS=20 timeout -k 10 120 $G a4 1769472 1024 1024 1 3 0
  go k3_walk_$r VP3D_NOCHECK=1 VP3D_ITERS=20 VP3D_A4_WALK=2 timeout -k 10 120 $G a4 1769472 1024 1024 1 3 0
done
go k3_walk_t VP3D_NOCHECK=1 VP3D_A4_WALK=2 timeout -k 10 120 $G a4t 1769472 1024 1024 1 3 0
echo done
