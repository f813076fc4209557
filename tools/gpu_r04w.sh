#!/bin/bash
# Round 4 step w: config 5, same box, the tree before the serve-end commit (tools/ab_old,
# a0d27c4) vs HEAD (serve form as its own instantiation), alternating; then the stream tests.
set -o pipefail
O=gpurun_out/r04w
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_stream.py -m gpu > $O/pytest_stream.txt 2>&1
rc=$?; tail -2 $O/pytest_stream.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  (cd tools/ab_old && timeout -k 10 300 python bench.py --stream --steps 4096 --warmup 256 --cpu-seconds 0) > $O/old_$r.log 2>&1 || exit 1
  echo "old: $(python -c "import json,sys; d=json.loads(open('$O/old_$r.log').read().strip().splitlines()[-1]); print(d['ms_per_step']*1e3, d['serve_latency_us'], d['eager_step_latency_us'])")"
  timeout -k 10 300 python bench.py --stream --steps 4096 --warmup 256 --cpu-seconds 0 > $O/new_$r.log 2>&1 || exit 1
  echo "new: $(python -c "import json,sys; d=json.loads(open('$O/new_$r.log').read().strip().splitlines()[-1]); print(d['ms_per_step']*1e3, d['serve_latency_us'], d['eager_step_latency_us'])")"
done
