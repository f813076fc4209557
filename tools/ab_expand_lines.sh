#!/bin/bash
# f16x3 expand: whole-line stores (DPP row_ror:8 trade between rows r and r + 8) vs the
# stores in flight at the chunk-end wait) vs the committed tree (tools/ab_old), same box
set -o pipefail
O=gpurun_out/abwl
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_lifter.py tests/test_gpu_golden.py tests/test_gpu_traj.py tests/test_gpu_pipeline.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for b in 65536 8192; do
    st=$([ $b = 8192 ] && echo 150 || echo 20)
    for v in new old; do
      d=.; [ $v = old ] && d=tools/ab_old
      timeout -k 10 200 python $d/bench.py --dtype f16x3 --batch $b --steps $st --warmup 5 --no-extras --no-legs > $O/b_${b}_${v}_$r.log 2>&1 || exit 1
      echo "${b}_${v}_$r: $(python tools/bench_brief.py $O/b_${b}_${v}_$r.log)"
    done
  done
done
timeout -k 10 300 python bench.py --traj --dtype f16x3 --steps 10 --warmup 3 --no-extras --no-legs > $O/traj_new.log 2>&1 && echo "traj_new: $(python tools/bench_brief.py $O/traj_new.log)"
timeout -k 10 300 python tools/ab_old/bench.py --traj --dtype f16x3 --steps 10 --warmup 3 --no-extras --no-legs > $O/traj_old.log 2>&1 && echo "traj_old: $(python tools/bench_brief.py $O/traj_old.log)"
