#!/bin/bash
# Round 4 step v: the other bench modes at HEAD -- sequence mode, training, the trajectory
# lifters, config 5 on its own (more steps than the default line's leg), config 3 as the main line.
set -o pipefail
O=gpurun_out/r04v
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --sequence --steps 10 --warmup 3 > $O/bench_sequence.log 2>&1 || exit 1
echo "seq:    $(tail -1 $O/bench_sequence.log | cut -c1-220)"
timeout -k 10 300 python bench.py --train --steps 5 --warmup 2 > $O/bench_train.log 2>&1 || exit 1
echo "train:  $(tail -1 $O/bench_train.log | cut -c1-220)"
timeout -k 10 300 python bench.py --seq-model transformer --steps 5 --warmup 2 > $O/bench_seq_transformer.log 2>&1 || exit 1
echo "tf:     $(tail -1 $O/bench_seq_transformer.log | cut -c1-220)"
timeout -k 10 300 python bench.py --seq-model lstm --steps 5 --warmup 2 > $O/bench_seq_lstm.log 2>&1 || exit 1
echo "lstm:   $(tail -1 $O/bench_seq_lstm.log | cut -c1-220)"
timeout -k 10 300 python bench.py --stream --steps 4096 --warmup 256 --cpu-seconds 5 > $O/bench_stream.log 2>&1 || exit 1
echo "stream: $(tail -1 $O/bench_stream.log | cut -c1-300)"
timeout -k 10 400 python bench.py --traj --steps 20 --warmup 5 > $O/bench_traj.log 2>&1 || exit 1
echo "traj:   $(python tools/bench_brief.py $O/bench_traj.log)"
