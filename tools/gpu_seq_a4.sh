#!/bin/bash
# Sequence mode (dilated k3 convs, taps d rows apart): conv_gemm_a4 forced (VP3D_GEMM=a4) vs the
# default LDS-ring kernel, bit identity vs q64 on the dilated layers (pytest), bench A/B.
set -o pipefail
TAG=${1:-seqa4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lifter.py -x -v -p no:cacheprovider --timeout 240 --timeout-method thread -k "dilated_seq_a4 or override" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && { tail -20 $OUT/pytest.log; exit $rc; }
B="python bench.py --sequence --steps 20 --warmup 5 --cpu-seconds 0"
for r in 1 2; do
  timeout -k 10 300 $B > $OUT/seq_def_$r.log 2>&1 || exit $?
  VP3D_GEMM=a4 timeout -k 10 300 $B > $OUT/seq_a4_$r.log 2>&1 || exit $?
  echo "def: $(python tools/bench_brief.py $OUT/seq_def_$r.log)"
  echo "a4:  $(python tools/bench_brief.py $OUT/seq_a4_$r.log)"
done
