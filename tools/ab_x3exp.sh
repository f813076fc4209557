#!/bin/bash
# X3 expand epilogue (packed BN, integer ReLU, DPP bank masks, buffer stores) vs the committed
# tree: bit identity of whole forwards (config 4 f16x3 at 65,536 and 8,192 windows, config 3),
# ablations, then alternating bench runs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_x3exp; mkdir -p $O
for cfg in "65536:" "8192:" "4096:--traj"; do
  b=${cfg%%:*}; ex=${cfg#*:}
  timeout -k 10 200 python tools/dump_forward.py $O/new_$b.npy --batch $b $ex > /dev/null 2>&1 || { echo "dump new $b failed"; exit 1; }
  timeout -k 10 200 python tools/ab_old/tools/dump_forward.py $O/old_$b.npy --batch $b $ex > /dev/null 2>&1 || { echo "dump old $b failed"; exit 1; }
  python -c "import numpy as np,sys; a=np.load('$O/new_$b.npy'); b=np.load('$O/old_$b.npy'); print('$b $ex bit-identical:', np.array_equal(a,b), 'max|d|', float(np.abs(a-b).max()))"
done
VP3D_X3=1 timeout -k 10 200 ./tools/ubench/expand_check 65536 0 0 2 16 18 || exit 1
bash tools/ab.sh x3exp "" "--dtype f16x3 --steps 20 --warmup 5 --no-extras --no-legs" 2
