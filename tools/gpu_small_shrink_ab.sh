#!/bin/bash
# f16x3 split shrink at small batches (64-row workgroups below 32,768 rows) vs the exact-f32
# shrink (VP3D_X3_SHRINK=f32: the narrow f32 kernel there): shrink / shard tests, then config 4
# at 8,192 and 1,024 windows alternating.  usage: bash tools/gpu_small_shrink_ab.sh [tag]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-smallshrink}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_lifter.py tests/test_gpu_shard.py -k "shrink or shard or eight or ranks or half_n" -x -v \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -15 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for m in split f32; do
    if [ $m = f32 ]; then export VP3D_X3_SHRINK=f32; else unset VP3D_X3_SHRINK; fi
    for b in 8192 1024; do
      timeout -k 10 200 python bench.py --no-extras --steps 40 --warmup 5 --global-batch $b > $O/b${b}_${m}_$r.log 2>&1 || { echo "bench $b $m failed"; tail -5 $O/b${b}_${m}_$r.log; exit 1; }
      echo "r${r}_${b}_$m: $(python tools/bench_brief.py $O/b${b}_${m}_$r.log)"
    done
  done
done
