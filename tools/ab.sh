#!/bin/bash
# Same-box A/B of the working tree ("new") against a committed tree built in tools/ab_old
# ("old": `git worktree add tools/ab_old <rev>` + its build, done on the CPU side first).
# Runs the given GPU tests once (new tree), then alternates new / old bench runs.
# usage: bash tools/ab.sh <tag> "<pytest paths or ''>" "<bench args>" [rounds]
#   e.g. bash tools/ab.sh x3epi "tests/test_gpu_lifter.py" "--dtype f16x3 --steps 20 --no-extras --no-legs" 2
set -o pipefail
tag=${1:?tag}; tests=$2; bargs=${3:?bench args}; rounds=${4:-2}
O=gpurun_out/ab_$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$tests" ]; then
  timeout -k 10 600 python -u -m pytest $tests -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for r in $(seq 1 $rounds); do
  for v in new old; do
    d=.; [ $v = old ] && d=tools/ab_old
    timeout -k 10 300 python $d/bench.py $bargs > $O/${v}_$r.log 2>&1 || { tail -5 $O/${v}_$r.log; exit 1; }
    echo "${v}_$r: $(python tools/bench_brief.py $O/${v}_$r.log)"
  done
done
