#!/bin/bash
# expand_gemm's split last round (VP3D_EXPAND_SPLIT=1, default) vs whole row blocks (0): config 4
# at 8,192 windows per GPU (N = 8's share), alternating, 3 repeats each
set -o pipefail
O=gpurun_out/abx2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  for dt in f16x3 bf16; do
    for sp in 1 0; do
      VP3D_EXPAND_SPLIT=$sp timeout -k 10 200 python bench.py --dtype $dt --batch 8192 --steps 200 --warmup 5 --no-extras --no-legs > $O/b_${dt}_s${sp}_$r.log 2>&1 || exit 1
      echo "${dt}_s${sp}_$r: $(python tools/bench_brief.py $O/b_${dt}_s${sp}_$r.log | cut -c1-120)"
    done
  done
done
