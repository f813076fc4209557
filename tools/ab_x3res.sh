#!/bin/bash
# X3 1x1 residual through LDS (working tree) vs the committed tree (tools/ab_old): GPU lifter /
# golden / traj tests, the ablation harness, then config 4 f16x3 alternating, same box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_x3res; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lifter.py tests/test_gpu_golden.py tests/test_gpu_traj.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for a in 0 8 16 32; do timeout -k 10 120 ./tools/ubench/x3_1x1_check 65536 $a || exit 1; done
bash tools/ab.sh x3res "" "--dtype f16x3 --steps 20 --warmup 5 --no-extras --no-legs" 2 || exit 1
bash tools/ab.sh x3res8k "" "--dtype f16x3 --batch 8192 --steps 100 --warmup 5 --no-extras --no-legs" 1
