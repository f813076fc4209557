#!/bin/bash
# f16x3 shrink in split fp16 (default since round 6) vs the exact-f32 shrink (VP3D_X3_SHRINK=f32):
# the shrink / shard / golden tests, then config 4 (no legs) and sequence mode alternating.
# usage: bash tools/gpu_x3_shrink_ab.sh [tag]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x3shrink}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lifter.py tests/test_gpu_shard.py tests/test_gpu_golden.py -k "shrink or shard or eight or ranks or golden or split_tail or config4" -x -v \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -15 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for m in split f32; do
    if [ $m = f32 ]; then export VP3D_X3_SHRINK=f32; else unset VP3D_X3_SHRINK; fi
    timeout -k 10 200 python bench.py --no-extras --steps 10 --warmup 3 > $O/c4_${m}_$r.log 2>&1 || { echo "bench c4 $m failed"; tail -5 $O/c4_${m}_$r.log; exit 1; }
    echo "r${r}_c4_$m: $(python tools/bench_brief.py $O/c4_${m}_$r.log)"
    timeout -k 10 200 python bench.py --sequence --dtype f16x3 --steps 10 --warmup 3 --cpu-seconds 0 > $O/seq_${m}_$r.log 2>&1 || { echo "bench seq $m failed"; tail -5 $O/seq_${m}_$r.log; exit 1; }
    echo "r${r}_seq_$m: $(python tools/bench_brief.py $O/seq_${m}_$r.log)"
  done
done
