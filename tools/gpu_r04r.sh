#!/bin/bash
# Round 4 step r: split-K restricted to long-K layers over few rounds (the f16x3 k3 convs) --
# parity, then B = 8,192 A/B (VP3D_A4_SPLIT 1 / 0) for f16x3 and bf16.
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_lifter.py tests/test_gpu_golden.py tests/test_gpu_traj.py tests/test_gpu_shard.py -m gpu > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for dt in f16x3 bf16; do
  for sp in 1 0; do
    VP3D_A4_SPLIT=$sp timeout -k 10 300 python bench.py --dtype $dt --global-batch 8192 --no-extras --steps 40 --warmup 5 > $O/b_${dt}_s${sp}_$r.log 2>&1 || exit 1
    echo "$dt split=$sp $(python tools/bench_brief.py $O/b_${dt}_s${sp}_$r.log)"
  done
done
done
