#!/bin/bash
# Green check at HEAD (one gpurun call): every -m gpu test, smoke(), the default bench line.
# Usage: bash tools/gpu_check.sh TAG   (outputs under gpurun_out/TAG)
set -o pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -5 $OUT/smoke.log; exit 1; }
echo "smoke: $(tail -1 $OUT/smoke.log)"
timeout -k 10 600 python bench.py > $OUT/bench_default.log 2>&1 || { echo bench failed; tail -5 $OUT/bench_default.log; exit 1; }
python tools/bench_brief.py $OUT/bench_default.log
