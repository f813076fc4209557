#!/bin/bash
# Round 4 step u: f16x3 expand with the chunk's stores deferred under the next chunk's MFMAs --
# parity, then a same-box A/B (VP3D_X3_DEFER 1 / 0) of the f16x3 config-4 and config-3 lines.
set -o pipefail
O=gpurun_out/r04u
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_lifter.py tests/test_gpu_golden.py tests/test_gpu_traj.py tests/test_gpu_pipeline.py -m gpu -k "x3 or f16x3 or fp32 or traj or golden or pipeline or window" > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for d in 1 0; do
    VP3D_X3_DEFER=$d timeout -k 10 300 python bench.py --dtype f16x3 --no-extras --steps 20 --warmup 5 > $O/b_d${d}_$r.log 2>&1 || exit 1
    echo "defer=$d $(python tools/bench_brief.py $O/b_d${d}_$r.log)"
  done
done
for d in 1 0; do
  VP3D_X3_DEFER=$d timeout -k 10 300 python bench.py --traj --dtype f16x3 --no-extras --steps 20 --warmup 5 > $O/t_d${d}.log 2>&1 || exit 1
  echo "traj defer=$d $(python tools/bench_brief.py $O/t_d${d}.log)"
done
