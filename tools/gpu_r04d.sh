#!/bin/bash
# Round 4 step d: the MFMA chains on the real block operands (config-4 and dolly windows).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r04d_mfma_bias_real.txt
: > $out
for spec in "1 " "3 " "1 --dolly"; do
  set -- $spec
  d=/tmp/ro_$1$2
  timeout -k 10 120 python -u tools/real_operands.py $d --block $1 $2 >> $out 2>&1 || exit 1
  echo "== block $1 $2 k3" >> $out
  timeout -k 10 120 tools/ubench/mfma_bias file $d/k3_A.bin $d/k3_W.bin 1024 1024 3072 >> $out 2>&1 || exit 1
  echo "== block $1 $2 1x1" >> $out
  timeout -k 10 120 tools/ubench/mfma_bias file $d/p_A.bin $d/p_W.bin 1024 1024 1024 >> $out 2>&1 || exit 1
done
cat $out
