set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/walk; mkdir -p $O
for r in 1 2; do
  for w in 1 0 2; do
    VP3D_A4_WALK=$w timeout -k 10 200 python bench.py --sequence --dtype f16x3 --steps 10 --warmup 3 --cpu-seconds 0 > $O/seq_w${w}_$r.log 2>&1 || { echo "seq w$w failed"; tail -5 $O/seq_w${w}_$r.log; exit 1; }
    echo "r${r}_seq_walk$w: $(python tools/bench_brief.py $O/seq_w${w}_$r.log)"
  done
done
