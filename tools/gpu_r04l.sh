#!/bin/bash
# Round 4 step l: f16x3 at B = 8,192 (config 4's per-GPU share at N = 8) and 65,536: per-layer
# times, a kernel trace at 8,192, and the MFMA-busy / clock PMC pass at 65,536.
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for B in 8192 16384 32768; do
  timeout -k 10 300 python bench.py --dtype f16x3 --global-batch $B --no-extras --steps 40 --warmup 5 > $O/b_f16x3_$B.log 2>&1 || exit 1
  echo "B=$B $(python tools/bench_brief.py $O/b_f16x3_$B.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8k -o run --output-format csv -- python bench.py --dtype f16x3 --global-batch 8192 --steps 20 --warmup 3 --no-extras > $O/prof8k.log 2>&1 || exit 1
echo prof8k ok
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $O/pmc_busy -o run -- python bench.py --dtype f16x3 --steps 3 --warmup 1 --no-extras --parity-windows 4 > $O/pmc_busy.log 2>&1 || exit 1
echo pmc ok
