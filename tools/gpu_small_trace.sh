#!/bin/bash
# Per-layer kernel trace at config 4's per-GPU shard at N = 8 (8,192 windows, f16x3 and bf16),
# beside the bench line itself.  usage: bash tools/gpu_small_trace.sh [tag]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-small}
mkdir -p $O
for dt in f16x3 bf16; do
  timeout -k 10 200 python bench.py --dtype $dt --global-batch 8192 --steps 20 --warmup 5 --cpu-seconds 0 --no-extras --no-legs > $O/bench_$dt.log 2>&1 || { echo "bench $dt failed"; tail -5 $O/bench_$dt.log; exit 1; }
  echo "$dt: $(python tools/bench_brief.py $O/bench_$dt.log)"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$dt -o run --output-format csv -- python bench.py --dtype $dt --global-batch 8192 --steps 10 --warmup 3 --cpu-seconds 0 --no-extras --no-legs > $O/prof_$dt.log 2>&1 || exit $?
done
echo done
