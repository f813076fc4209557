#!/bin/bash
# N-rank bench path rehearsed on a 1-GPU box (VP3D_BENCH_REHEARSE=1: ranks share the device,
# gloo instead of RCCL) + kernel trace of the config-5 stream bench.
set -o pipefail
OUT=gpurun_out/${1:-rehearse}
mkdir -p $OUT
export TMPDIR=/tmp
VP3D_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $OUT/bench_n2.log 2>&1 || exit $?
echo "n2: $(tail -1 $OUT/bench_n2.log | cut -c1-400)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_stream -o run --output-format csv -- \
  python bench.py --stream --steps 4096 --warmup 128 --cpu-seconds 5 > $OUT/bench_stream.log 2>&1 || exit $?
echo "stream: $(tail -1 $OUT/bench_stream.log | cut -c1-600)"
