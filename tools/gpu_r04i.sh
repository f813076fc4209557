#!/bin/bash
# Round 4 step i: one split-fp16 layer through the library's q64 / a4 X3 kernels on real block
# operands (config-4 windows blocks 1 and 3, dolly block 1), against exact sums.
set -o pipefail
mkdir -p gpurun_out/r04i
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r04i/x3_layer_check.txt
: > $o
for spec in "1 " "3 " "1 --dolly"; do
  set -- $spec
  d=/tmp/ro_$1$2
  timeout -k 10 120 python -u tools/real_operands.py $d --block $1 $2 >> $o 2>&1 || exit 1
  echo "== block $1 $2 k3" >> $o
  timeout -k 10 120 tools/ubench/x3_layer_check $d/k3_A.bin $d/k3_W.bin 1024 1024 3072 >> $o 2>&1 || exit 1
  echo "== block $1 $2 1x1" >> $o
  timeout -k 10 120 tools/ubench/x3_layer_check $d/p_A.bin $d/p_W.bin 1024 1024 1024 >> $o 2>&1 || exit 1
done
cat $o
