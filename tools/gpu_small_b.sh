#!/bin/bash
# Green check at HEAD plus the small-batch picture (config 4 at N = 8 is 8,192 windows per GPU):
# kernel traces of the bf16 bench at B = 8,192 with the default dispatch and with the
# 128x128 kernel everywhere (VP3D_GEMM=h16), for the per-layer tile-count comparison.
# Usage: bash tools/gpu_small_b.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-smallb}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(tail -1 $OUT/$name.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then tail -8 $OUT/$name.log; exit $rc; fi
}
if [ -z "$2" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
  run smoke 120 python __graft_entry__.py smoke
fi
B="python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --parity-windows 4 --no-extras --global-batch 8192"
run bench_8k 300 $B
run trace_8k 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_8k -o run --output-format csv -- $B
run trace_8k_h16 300 env VP3D_GEMM=h16 rocprofv3 --kernel-trace --stats -d $OUT/trace_8k_h16 -o run --output-format csv -- $B
echo done
