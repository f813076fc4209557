#!/bin/bash
# Round-3 profile session (one gpurun call): the default bench line (as the driver runs it),
# rocprofv3 kernel traces of the headline bench
# (bf16), the fp32 and f16x3 legs alone, and the config-5 stream; PMC passes (counters
# only, one pass each): FETCH_SIZE / WRITE_SIZE for bf16 and f16x3, MFMA-busy and
# instruction-wait cycles for bf16; FETCH / WRITE for the stream.
# Usage: bash tools/gpu_profiles_r03.sh TAG   (outputs under gpurun_out/TAG)
set -o pipefail
TAG=${1:-r03prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
}
run bench_default 600 python bench.py
B="python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --parity-windows 4 --no-extras"
run trace_bf16 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_bf16 -o run --output-format csv -- $B
run trace_fp32 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_fp32 -o run --output-format csv -- $B --dtype fp32
run trace_x3 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_x3 -o run --output-format csv -- $B --dtype f16x3
for C in FETCH_SIZE WRITE_SIZE; do
  run pmc_bf16_$C 300 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_bf16_$C -o run -- $B
  run pmc_x3_$C 300 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_x3_$C -o run -- $B --dtype f16x3
done
run pmc_bf16_busy 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_bf16_busy -o run -- $B
S="python bench.py --stream --steps 1024 --warmup 64 --cpu-seconds 0"
run trace_stream 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_stream -o run --output-format csv -- $S
for C in FETCH_SIZE WRITE_SIZE; do
  run pmc_stream_$C 300 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_stream_$C -o run -- $S
done
echo done
