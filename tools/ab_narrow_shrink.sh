#!/bin/bash
# exact-f32 shrink: the narrow kernel with an 8-step operand ring (new) vs 1 step (tools/ab_old),
# and vs the 128x128 tile kernel (VP3D_F32_NARROW=0); at 65,536 windows the narrow kernel forced
# (VP3D_F32_NARROW=2) vs the tile kernel (default there); f16x3 config 4, same box
set -o pipefail
O=gpurun_out/abns
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_lifter.py -k "narrow or opt1f_243_fp32 or config4" -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in new old tile; do
    d=.; [ $v = old ] && d=tools/ab_old
    e=1; [ $v = tile ] && e=0
    VP3D_F32_NARROW=$e timeout -k 10 200 python $d/bench.py --dtype f16x3 --batch 8192 --steps 100 --warmup 5 --no-extras --no-legs > $O/b8_${v}_$r.log 2>&1 || exit 1
    echo "8192_${v}_$r: $(python tools/bench_brief.py $O/b8_${v}_$r.log | grep -o 'shrink=[0-9.]*') $(python tools/bench_brief.py $O/b8_${v}_$r.log | cut -c1-40)"
  done
  for e in 1 2; do
    VP3D_F32_NARROW=$e timeout -k 10 200 python bench.py --dtype f16x3 --steps 15 --warmup 3 --no-extras --no-legs > $O/b64_e${e}_$r.log 2>&1 || exit 1
    echo "65536_narrow${e}_$r: $(python tools/bench_brief.py $O/b64_e${e}_$r.log | grep -o 'shrink=[0-9.]*') $(python tools/bench_brief.py $O/b64_e${e}_$r.log | cut -c1-40)"
  done
done
