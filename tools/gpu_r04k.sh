#!/bin/bash
# Round 4 step k: a4 grouped LDS-DMA pieces (one M0 per 4 pieces) -- bit identity vs q64 and the
# goldens, then a same-box A/B of the default bench (bf16 and f16x3) with VP3D_A4_GD=1 / 0.
set -o pipefail
O=gpurun_out/r04k
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_lifter.py tests/test_gpu_golden.py tests/test_gpu_traj.py -m gpu > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for gd in 1 0; do
    for dt in bf16 f16x3; do
      VP3D_A4_GD=$gd timeout -k 10 300 python bench.py --dtype $dt --no-extras --steps 20 --warmup 5 > $O/b_${dt}_gd${gd}_$r.log 2>&1 || exit 1
      echo "gd=$gd $(python tools/bench_brief.py $O/b_${dt}_gd${gd}_$r.log)"
    done
  done
done
