#!/bin/bash
# Round 4 step s: the green check at HEAD -- every -m gpu test, smoke(), the default bench line,
# and a rocprofv3 kernel trace of the default (f16x3) config-4 line.
set -o pipefail
OUT=gpurun_out/r04s
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -5 $OUT/smoke.log; exit 1; }
echo "smoke: $(tail -1 $OUT/smoke.log)"
timeout -k 10 600 python bench.py > $OUT/bench_default.log 2>&1 || { echo bench failed; tail -5 $OUT/bench_default.log; exit 1; }
python tools/bench_brief.py $OUT/bench_default.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-extras > $OUT/prof.log 2>&1 || exit $?
echo "prof ok"
