#!/bin/bash
# f16x3 expand: nontemporal (default) vs cached stores (VP3D_X3_EXPAND_NT=0), config 3 and 4
set -o pipefail
O=gpurun_out/abnt
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for nt in 1 0; do
    VP3D_X3_EXPAND_NT=$nt timeout -k 10 300 python bench.py --traj --dtype f16x3 --steps 15 --warmup 3 --no-extras --no-legs > $O/t_nt${nt}_$r.log 2>&1 || exit 1
    echo "traj_nt${nt}_$r: $(python tools/bench_brief.py $O/t_nt${nt}_$r.log)"
    VP3D_X3_EXPAND_NT=$nt timeout -k 10 300 python bench.py --dtype f16x3 --steps 15 --warmup 3 --no-extras --no-legs > $O/c4_nt${nt}_$r.log 2>&1 || exit 1
    echo "c4_nt${nt}_$r: $(python tools/bench_brief.py $O/c4_nt${nt}_$r.log)"
  done
done
