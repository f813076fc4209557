#!/bin/bash
# split-K tails and the f16x3 shrink with 64-row workgroups (default) vs 256-row ones
# (VP3D_TAIL_RBW=4): tail / shrink / shard tests, then sequence mode (f16x3, bf16) and config 4
# alternating.  usage: bash tools/gpu_tail_rbw_ab.sh [tag]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-rbw}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_lifter.py tests/test_gpu_shard.py -k "shrink or shard or eight or ranks or tail or seq" -x -v \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -15 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for m in 1 4; do
    export VP3D_TAIL_RBW=$m
    for dt in f16x3 bf16; do
      timeout -k 10 200 python bench.py --sequence --dtype $dt --steps 10 --warmup 3 --cpu-seconds 0 > $O/seq_${dt}_${m}_$r.log 2>&1 || { echo "seq $dt $m failed"; tail -5 $O/seq_${dt}_${m}_$r.log; exit 1; }
      echo "r${r}_seq_${dt}_rbw$m: $(python tools/bench_brief.py $O/seq_${dt}_${m}_$r.log)"
    done
    timeout -k 10 200 python bench.py --no-extras --steps 10 --warmup 3 > $O/c4_${m}_$r.log 2>&1 || { echo "c4 $m failed"; exit 1; }
    echo "r${r}_c4_rbw$m: $(python tools/bench_brief.py $O/c4_${m}_$r.log)"
  done
done
