#!/bin/bash
# One GPU session: parity tests, the bench configurations, a rocprofv3 kernel trace
# of the headline bench and the FETCH_SIZE / WRITE_SIZE PMC passes (separate runs,
# counters only) that tools/traffic.py turns into per-layer HBM bytes (headline and
# trajectory configurations).
# Usage: [HEAD_ONLY=1 | TAIL_ONLY=1] bash tools/gpu_round.sh TAG  (HEAD: tests, benches,
# profiles; TAIL: training / sequence-model / sequence benches and the smoke run)
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$TAIL_ONLY" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench_bf16.log 2>&1 || exit $?
echo "bf16:   $(python tools/bench_brief.py $OUT/bench_bf16.log)"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --dtype fp16 --no-extras > $OUT/bench_fp16.log 2>&1 || exit $?
echo "fp16:   $(python tools/bench_brief.py $OUT/bench_fp16.log)"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --traj --no-extras > $OUT/bench_traj.log 2>&1 || exit $?
echo "traj:   $(python tools/bench_brief.py $OUT/bench_traj.log)"
timeout -k 10 300 python bench.py --stream --steps 4096 --warmup 128 --cpu-seconds 5 > $OUT/bench_stream.log 2>&1 || exit $?
echo "stream: $(tail -1 $OUT/bench_stream.log | cut -c1-300)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-extras > $OUT/prof.log 2>&1 || exit $?
echo "prof ok"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o run -- python bench.py --steps 3 --warmup 1 --no-extras --parity-windows 4 > $OUT/pmc_$C.log 2>&1 || exit $?
  echo "pmc $C ok"
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $OUT/traj_pmc_$C -o run -- python bench.py --traj --steps 3 --warmup 1 --no-extras --parity-windows 4 > $OUT/traj_pmc_$C.log 2>&1 || exit $?
  echo "traj pmc $C ok"
done
fi
if [ -n "$HEAD_ONLY" ]; then exit 0; fi
timeout -k 10 300 python bench.py --train --steps 5 --warmup 2 > $OUT/bench_train.log 2>&1 || exit $?
echo "train:  $(tail -1 $OUT/bench_train.log | cut -c1-200)"
timeout -k 10 300 python bench.py --seq-model transformer --steps 5 --warmup 2 > $OUT/bench_seq_transformer.log 2>&1 || exit $?
echo "tf:     $(tail -1 $OUT/bench_seq_transformer.log | cut -c1-200)"
timeout -k 10 300 python bench.py --seq-model lstm --steps 5 --warmup 2 > $OUT/bench_seq_lstm.log 2>&1 || exit $?
echo "lstm:   $(tail -1 $OUT/bench_seq_lstm.log | cut -c1-200)"
timeout -k 10 300 python bench.py --sequence --steps 10 --warmup 3 > $OUT/bench_sequence.log 2>&1 || exit $?
echo "seq:    $(tail -1 $OUT/bench_sequence.log | cut -c1-200)"
timeout -k 10 120 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || exit $?
echo "smoke:  $(tail -1 $OUT/smoke.log)"
