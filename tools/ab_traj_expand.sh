#!/bin/bash
# config 3 f16x3 expand (camera concat, NKS = 5): scale / shift from global memory (two
# workgroups per CU) with half-line (new) or whole-line (tools/ab_b) stores vs the committed
# tree (tools/ab_old: LDS scale / shift, one workgroup per CU), same box
set -o pipefail
O=gpurun_out/abtx
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_traj.py tests/test_gpu_golden.py tests/test_gpu_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in new b old; do
    d=.; [ $v = old ] && d=tools/ab_old; [ $v = b ] && d=tools/ab_b
    timeout -k 10 300 python $d/bench.py --traj --dtype f16x3 --steps 15 --warmup 3 --no-extras --no-legs > $O/t_${v}_$r.log 2>&1 || exit 1
    echo "${v}_$r: $(python tools/bench_brief.py $O/t_${v}_$r.log)"
  done
done
