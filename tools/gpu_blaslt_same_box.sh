#!/bin/bash
# hipBLASLt (torch.matmul, bf16) vs conv_gemm_a4 on the block-1 k3 shape at B = 65,536, same
# box, post-ReLU A operand for both: torch, a4 (strided, gemm_check), torch again.
set -o pipefail
TAG=${1:-blaslt}
OUT=gpurun_out/$TAG
mkdir -p $OUT
go() {  # name, env/command...
  local name=$1; shift
  env "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(grep -E 'TFLOP|bad=' $OUT/$name.log | tr '\n' ' ' | cut -c1-600)"
  [ $rc -ne 0 ] && exit $rc
}
go torch_1 TORCH_GEMM_B=65536 TORCH_GEMM_RELU=1 timeout -k 10 180 python tools/ubench/torch_gemm.py
go a4_k3 VP3D_STRIDE=3 VP3D_NOCHECK=1 VP3D_RELU_A=1 VP3D_ITERS=20 timeout -k 10 150 tools/ubench/gemm_check a4 1769472 1024 1024 1 3 0
go a4_1x1 VP3D_NOCHECK=1 VP3D_RELU_A=1 VP3D_ITERS=20 timeout -k 10 150 tools/ubench/gemm_check a4 1769472 1024 1024 1 1 1
go torch_2 TORCH_GEMM_B=65536 TORCH_GEMM_RELU=1 timeout -k 10 180 python tools/ubench/torch_gemm.py
echo done
