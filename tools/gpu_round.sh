#!/bin/bash
# One GPU session: parity tests, then benches, then a rocprofv3 kernel-trace of the bench.
# Usage (on the GPU box, from the repo root): bash tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -s -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 "$@" > $OUT/bench_bf16.log 2>&1 || exit $?
tail -1 $OUT/bench_bf16.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --dtype fp32 --cpu-seconds 0 "$@" > $OUT/bench_fp32.log 2>&1 || exit $?
tail -1 $OUT/bench_fp32.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-seconds 0 "$@" > $OUT/prof.log 2>&1 || exit $?
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -c1-200 {} | head -12'
