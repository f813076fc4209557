#!/bin/bash
# bf16 at 8,192 windows per GPU: every layer on the 128x128 kernel (VP3D_GEMM=h16) vs the
# default dispatch -- per-layer times for the small blocks (3-4) whose 256x256 tiles leave
# partial rounds
set -o pipefail
O=gpurun_out/abst
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for g in default h16; do
    if [ $g = h16 ]; then export VP3D_GEMM=h16; else unset VP3D_GEMM; fi
    timeout -k 10 200 python bench.py --dtype bf16 --batch 8192 --steps 150 --warmup 5 --no-extras --no-legs > $O/b_${g}_$r.log 2>&1 || exit 1
    echo "${g}_$r: $(python tools/bench_brief.py $O/b_${g}_$r.log)"
  done
done
