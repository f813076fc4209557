#!/bin/bash
# Round-3 refresh of the secondary configurations at HEAD: config 3 (trajectory, fp16 + f16x3
# leg), config 5 stream, sequence mode, training, the two trajectory lifters, fp16 config 4.
set -o pipefail
TAG=${1:-r03tail}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(tail -1 $OUT/$name.log | cut -c1-220)"
  if [ $rc -ne 0 ]; then tail -8 $OUT/$name.log; exit $rc; fi
}
run bench_traj 300 python bench.py --traj --steps 20 --warmup 5 --cpu-seconds 5
run bench_fp16 300 python bench.py --dtype fp16 --steps 20 --warmup 5 --no-extras
run bench_stream 300 python bench.py --stream --steps 4096 --warmup 128 --cpu-seconds 5
run bench_sequence 300 python bench.py --sequence --steps 10 --warmup 3 --cpu-seconds 5
run bench_train 300 python bench.py --train --steps 5 --warmup 2 --cpu-seconds 5
run bench_seq_transformer 300 python bench.py --seq-model transformer --steps 5 --warmup 2 --cpu-seconds 5
run bench_seq_lstm 300 python bench.py --seq-model lstm --steps 5 --warmup 2 --cpu-seconds 5
echo done
