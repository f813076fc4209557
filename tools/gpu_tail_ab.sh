#!/bin/bash
# Sequence-mode split-K tails (conv_gemm_tail.hip) on one box: the tail tests, then the
# f16x3 sequence bench with the split tails (default) and the quarter-N tiles (VP3D_A4_TAIL=hn)
# alternating, then a kernel trace of the default.  usage: bash tools/gpu_tail_ab.sh [tag]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-tail}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lifter.py -k "seq or tail" -x -v -p no:cacheprovider \
  --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -15 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for dt in f16x3 bf16; do
    for m in split hn; do
      if [ $m = hn ]; then export VP3D_A4_TAIL=hn; else unset VP3D_A4_TAIL; fi
      timeout -k 10 200 python bench.py --sequence --dtype $dt --steps 10 --warmup 3 --cpu-seconds 0 > $O/seq_${dt}_${m}_$r.log 2>&1 || { echo "bench $dt $m failed"; tail -5 $O/seq_${dt}_${m}_$r.log; exit 1; }
      echo "r${r}_${dt}_$m: $(python tools/bench_brief.py $O/seq_${dt}_${m}_$r.log)"
    done
  done
done
unset VP3D_A4_TAIL
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --sequence --dtype f16x3 --steps 5 --warmup 2 --cpu-seconds 0 > $O/prof.log 2>&1 || exit $?
echo prof ok
