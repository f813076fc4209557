#!/bin/bash
# Round 4 step m: split-fp16 epilogues on mixed-precision FMAs (v_fma_mix_f32 residual sums,
# v_fma_mixlo/mixhi_f16 lo halves) -- parity / bit identity, then the f16x3 and bf16 lines.
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_lifter.py tests/test_gpu_golden.py tests/test_gpu_traj.py tests/test_gpu_shard.py -m gpu > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for dt in f16x3 bf16; do
    timeout -k 10 300 python bench.py --dtype $dt --no-extras --steps 20 --warmup 5 > $O/b_${dt}_$r.log 2>&1 || exit 1
    echo "$(python tools/bench_brief.py $O/b_${dt}_$r.log)"
  done
done
timeout -k 10 300 python -u tools/x3_depth.py --B 512 --dtypes fp32,f16x3 > $O/x3_depth.txt 2>&1 || exit 1
tail -1 $O/x3_depth.txt
