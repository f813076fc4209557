#!/bin/bash
# 16-bit expand, camera-concat shape (K = 138, 5 k-slabs): RB 4 with a 2-chunk weight ring
# (72 KB LDS, two workgroups per CU; new) vs RB 2 with a 3-chunk ring (tools/ab_old); config 3
# fp16 main line, same box
set -o pipefail
O=gpurun_out/abc4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_traj.py tests/test_gpu_pipeline.py tests/test_gpu_golden.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in new old; do
    d=.; [ $v = old ] && d=tools/ab_old
    timeout -k 10 300 python $d/bench.py --traj --steps 20 --warmup 5 --no-extras --no-legs > $O/t_${v}_$r.log 2>&1 || exit 1
    echo "${v}_$r: $(python tools/bench_brief.py $O/t_${v}_$r.log)"
  done
done
