#!/bin/bash
# Round 4 step p: exact-f32 narrow GEMM for the shrink -- bit identity vs the tile kernel, parity,
# and the f16x3 line at B = 8,192 and 65,536.
set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_lifter.py tests/test_gpu_golden.py tests/test_gpu_seq_lifter.py tests/test_run_eval_seq.py tests/test_gpu_train.py -m gpu > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
for B in 8192 65536; do
  for nw in 1 0; do
    VP3D_F32_NARROW=$nw timeout -k 10 300 python bench.py --dtype f16x3 --global-batch $B --no-extras --steps 20 --warmup 5 > $O/b_${B}_n$nw.log 2>&1 || exit 1
    echo "B=$B narrow=$nw $(python tools/bench_brief.py $O/b_${B}_n$nw.log)"
  done
done
