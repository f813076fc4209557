#!/bin/bash
# config 5: the shrink folded into the last block's 1x1 (default) vs VP3D_STREAM_FOLD=0, same box:
# the stream tests, then --stream fp32 / fp16 lines alternating (pipelined step, serve p50/p99)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_fold; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for dt in fp32 fp16; do for f in 1 0; do
  VP3D_STREAM_FOLD=$f timeout -k 10 200 python bench.py --stream --dtype $dt --steps 4096 --warmup 256 --cpu-seconds 0 > $O/${dt}_f${f}_$r.log 2>&1 || { tail -5 $O/${dt}_f${f}_$r.log; exit 1; }
  python -c "
import json; d=json.loads(open('$O/${dt}_f${f}_$r.log').read().strip().split('\n')[-1])
print('$dt fold=$f r$r', 'step_us', d['roofline']['avg_step_us'], 'serve', d['serve_latency_us'], 'parity', {k: round(v, 7) for k, v in d['parity'].items() if 'delta' in k})"
done; done; done
