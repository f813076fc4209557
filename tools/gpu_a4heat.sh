#!/bin/bash
# conv_gemm_a4 on the B = 65,536 block-1 k3 shape: short vs long (heated) runs, random vs
# ReLU-output A operand -- where the harness (7.96 ms) and the bench (8.6 ms) part.
set -o pipefail
TAG=${1:-a4heat}
OUT=gpurun_out/$TAG
mkdir -p $OUT
G=tools/ubench/gemm_check
M=1769472
export VP3D_NOCHECK=1
go() {  # name, env..., -- args
  local name=$1; shift
  env "$@" > $OUT/$name.log 2>&1 || exit $?
  echo "$name: $(tail -1 $OUT/$name.log)"
}
go short       timeout -k 10 120 $G a4 $M 1024 1024 1 3 0
go long        VP3D_WARM=60 VP3D_ITERS=60 timeout -k 10 200 $G a4 $M 1024 1024 1 3 0
go relu_short  VP3D_RELU_A=1 timeout -k 10 120 $G a4 $M 1024 1024 1 3 0
go relu_long   VP3D_RELU_A=1 VP3D_WARM=60 VP3D_ITERS=60 timeout -k 10 200 $G a4 $M 1024 1024 1 3 0
go q64_long    VP3D_WARM=60 VP3D_ITERS=60 timeout -k 10 200 $G q64 $M 1024 1024 1 3 0
