#!/bin/bash
# Round-3 evidence at HEAD (one gpurun call): every -m gpu test, smoke(), the default bench
# line (as the driver runs it), a rocprofv3 kernel trace of the headline bench (bf16) and of
# the f16x3 leg, PMC FETCH_SIZE / WRITE_SIZE passes (bf16) for the committed traffic summary,
# and the MFMA-busy / issue-wait / clock pass.
# Usage: bash tools/gpu_final_r03.sh TAG   (outputs under gpurun_out/TAG)
set -o pipefail
TAG=${1:-r03final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(tail -1 $OUT/$name.log | cut -c1-160)"
  if [ $rc -ne 0 ]; then tail -8 $OUT/$name.log; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
run smoke 120 python __graft_entry__.py smoke
run bench_default 600 python bench.py
B="python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --parity-windows 4 --no-extras"
run trace_bf16 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_bf16 -o run --output-format csv -- $B
run trace_x3 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_x3 -o run --output-format csv -- $B --dtype f16x3
for C in FETCH_SIZE WRITE_SIZE; do
  run pmc_bf16_$C 300 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_bf16_$C -o run -- $B
done
run pmc_bf16_busy 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_bf16_busy -o run -- $B
echo done
