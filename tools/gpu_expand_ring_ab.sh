#!/bin/bash
# f16x3 expand, three workgroups per CU (VP3D_X3_EXPAND_RING=1: one resident weight chunk, RB 2)
# vs the default (2-chunk ring, RB 3, two per CU): bit identity of the forwards, then the config-4
# line without legs alternating.  usage: bash tools/gpu_expand_ring_ab.sh [tag]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ring}
mkdir -p $O
for b in 65536 8192; do
  timeout -k 10 200 python tools/dump_forward.py $O/d_$b.npy --batch $b > $O/dump_$b.log 2>&1 || { echo "dump failed"; tail -5 $O/dump_$b.log; exit 1; }
  VP3D_X3_EXPAND_RING=1 timeout -k 10 200 python tools/dump_forward.py $O/r_$b.npy --batch $b > $O/dumpr_$b.log 2>&1 || { echo "dump ring failed"; tail -5 $O/dumpr_$b.log; exit 1; }
  python -c "import numpy as np; a=np.load('$O/d_$b.npy'); b=np.load('$O/r_$b.npy'); print('B=$b bit-identical:', np.array_equal(a, b), float(np.abs(a-b).max()))"
done
for r in 1 2; do
  for m in def ring; do
    if [ $m = ring ]; then export VP3D_X3_EXPAND_RING=1; else unset VP3D_X3_EXPAND_RING; fi
    timeout -k 10 200 python bench.py --no-extras --steps 10 --warmup 3 > $O/c4_${m}_$r.log 2>&1 || { echo "bench $m failed"; tail -5 $O/c4_${m}_$r.log; exit 1; }
    echo "r${r}_c4_$m: $(python tools/bench_brief.py $O/c4_${m}_$r.log)"
    timeout -k 10 200 python bench.py --no-extras --steps 20 --warmup 3 --global-batch 8192 > $O/c8k_${m}_$r.log 2>&1 || { echo "bench 8k $m failed"; tail -5 $O/c8k_${m}_$r.log; exit 1; }
    echo "r${r}_8k_$m: $(python tools/bench_brief.py $O/c8k_${m}_$r.log)"
  done
done
