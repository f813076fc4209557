#!/bin/bash
# Round 4 step g: split-fp16 numerics (MFMA chain bias on synthetic and real dolly operands,
# output scale per dtype on the dolly and config-4 windows, per depth), then the green check.
set -o pipefail
OUT=gpurun_out/r04g
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=$OUT/numerics.txt
: > $o
timeout -k 10 60 tools/ubench/mfma_rounding >> $o 2>&1 &&
timeout -k 10 60 tools/ubench/cvt_rounding >> $o 2>&1 &&
for d in 0 2; do timeout -k 10 120 tools/ubench/mfma_bias 3072 512 $d >> $o 2>&1 || exit 1; done &&
timeout -k 10 120 python -u tools/real_operands.py /tmp/ro_d1 --block 1 --dolly >> $o 2>&1 &&
timeout -k 10 120 tools/ubench/mfma_bias file /tmp/ro_d1/k3_A.bin /tmp/ro_d1/k3_W.bin 1024 1024 3072 >> $o 2>&1 &&
timeout -k 10 120 tools/ubench/mfma_bias file /tmp/ro_d1/p_A.bin /tmp/ro_d1/p_W.bin 1024 1024 1024 >> $o 2>&1 &&
timeout -k 10 300 python -u tools/x3_shrink.py --B 256 --dtypes fp32,f16x3,fp16 >> $o 2>&1 &&
timeout -k 10 300 python -u tools/x3_shrink.py --B 256 --config4 --dtypes fp32,f16x3,fp16 >> $o 2>&1
rc=$?
cat $o
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_r04f.sh
