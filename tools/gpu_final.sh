#!/bin/bash
# The round's evidence runs on one MI355X box (run through gpurun, one stage per call):
#   check  -- every -m gpu test, smoke(), the default bench line, and a rocprofv3 kernel trace
#             of the default (f16x3, config 4) line                     -> gpurun_out/final/check
#   pmc    -- FETCH_SIZE / WRITE_SIZE passes (one counter per run) for the bench legs' launches:
#             config 4 f16x3 / bf16 / fp32, config 3 fp16 / f16x3 / fp32 -> gpurun_out/final/pmc
#             (tools/traffic.py turns them into profiles/traffic_*_b65536*.json)
#   modes  -- the other bench modes: config 3 as the main line, config 5 on its own, sequence
#             mode, training, the trajectory lifters                    -> gpurun_out/final/modes
# usage: bash tools/gpu_final.sh check|pmc|modes
set -o pipefail
stage=${1:?stage: check, pmc or modes}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final/$stage
mkdir -p $O
case $stage in
check)
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 120 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
  echo "smoke: $(tail -1 $O/smoke.log)"
  timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || { echo bench failed; tail -5 $O/bench_default.log; exit 1; }
  python tools/bench_brief.py $O/bench_default.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-extras > $O/prof.log 2>&1 || exit $?
  echo "prof ok"
  ;;
pmc)
  for spec in "f16x3:" "bf16:" "fp32:" "fp16:--traj" "f16x3:--traj" "fp32:--traj"; do
    dt=${spec%%:*}; ex=${spec#*:}; tag=${dt}${ex:+_traj}
    for C in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $O/$tag/pmc_$C -o run -- python bench.py --dtype $dt $ex --steps 3 --warmup 1 --no-extras --parity-windows 4 --settle-seconds 0.1 > $O/${tag}_$C.log 2>&1 || { echo "$tag $C failed"; tail -3 $O/${tag}_$C.log; exit 1; }
      echo "$tag $C ok"
    done
  done
  ;;
modes)
  timeout -k 10 400 python bench.py --traj --steps 20 --warmup 5 > $O/bench_traj.log 2>&1 || exit 1
  echo "traj:   $(python tools/bench_brief.py $O/bench_traj.log)"
  timeout -k 10 300 python bench.py --stream --steps 4096 --warmup 256 --cpu-seconds 5 > $O/bench_stream.log 2>&1 || exit 1
  echo "stream: $(tail -1 $O/bench_stream.log | cut -c1-300)"
  timeout -k 10 300 python bench.py --sequence --steps 10 --warmup 3 > $O/bench_sequence.log 2>&1 || exit 1
  echo "seq:    $(tail -1 $O/bench_sequence.log | cut -c1-220)"
  timeout -k 10 300 python bench.py --train --steps 5 --warmup 2 > $O/bench_train.log 2>&1 || exit 1
  echo "train:  $(tail -1 $O/bench_train.log | cut -c1-220)"
  timeout -k 10 300 python bench.py --seq-model transformer --steps 5 --warmup 2 > $O/bench_seq_transformer.log 2>&1 || exit 1
  echo "tf:     $(tail -1 $O/bench_seq_transformer.log | cut -c1-220)"
  timeout -k 10 300 python bench.py --seq-model lstm --steps 5 --warmup 2 > $O/bench_seq_lstm.log 2>&1 || exit 1
  echo "lstm:   $(tail -1 $O/bench_seq_lstm.log | cut -c1-220)"
  ;;
*) echo "unknown stage $stage"; exit 2 ;;
esac
