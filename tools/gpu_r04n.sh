#!/bin/bash
# Round 4 step n: the split-fp16 1x1 + residual layers walk their tiles -- parity / bit identity
# (walk on, off, every layer), then a same-box A/B of the f16x3 line (VP3D_A4_WALK 1 / 0).
set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_lifter.py tests/test_gpu_golden.py tests/test_gpu_traj.py tests/test_gpu_shard.py -m gpu > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for w in 1 0; do
    VP3D_A4_WALK=$w timeout -k 10 300 python bench.py --dtype f16x3 --no-extras --steps 20 --warmup 5 > $O/b_w${w}_$r.log 2>&1 || exit 1
    echo "walk=$w $(python tools/bench_brief.py $O/b_w${w}_$r.log)"
  done
done
