#!/bin/bash
# conv_gemm_a4 vs q64 on the STRIDED block-1 k3 shape (VP3D_STRIDE=3: input rows 3m .. 3m + 2,
# the Optimized1f layer's access pattern; the default harness shape is a stride-1 conv whose
# output rows share input rows): parity at B = 8,192, time and stamps at B = 65,536.
set -o pipefail
TAG=${1:-a4s3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
G=tools/ubench/gemm_check
export VP3D_STRIDE=3
go() {  # name, env/command...
  local name=$1; shift
  env "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(grep -E 'trace: (wave|kernel)|TFLOP|max\|d\|' $OUT/$name.log | tr '\n' ' ' | cut -c1-300)"
  [ $rc -ne 0 ] && exit $rc
}
go check_a4_8k timeout -k 10 120 $G a4 221184 1024 1024 1 3 0
go a4_65k   VP3D_NOCHECK=1 VP3D_RELU_A=1 timeout -k 10 120 $G a4 1769472 1024 1024 1 3 0
go q64_65k  VP3D_NOCHECK=1 VP3D_RELU_A=1 timeout -k 10 120 $G q64 1769472 1024 1024 1 3 0
go a4t_65k  VP3D_NOCHECK=1 VP3D_RELU_A=1 timeout -k 10 120 $G a4t 1769472 1024 1024 1 3 0
go a4abl1   VP3D_NOCHECK=1 VP3D_RELU_A=1 VP3D_ABL=1 timeout -k 10 120 $G a4 1769472 1024 1024 1 3 0
go a4abl3   VP3D_NOCHECK=1 VP3D_RELU_A=1 VP3D_ABL=3 timeout -k 10 120 $G a4 1769472 1024 1024 1 3 0
