#!/bin/bash
# Round 4 step t: FETCH_SIZE / WRITE_SIZE PMC passes (separate runs, counters only) for the
# bench legs' dominant launches: config 4 f16x3 / bf16 / fp32 and config 3 fp16 / f16x3 / fp32.
set -o pipefail
OUT=gpurun_out/r04t
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in "f16x3:" "bf16:" "fp32:" "fp16:--traj" "f16x3:--traj" "fp32:--traj"; do
  dt=${spec%%:*}; ex=${spec#*:}; tag=${dt}${ex:+_traj}
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $OUT/$tag/pmc_$C -o run -- python bench.py --dtype $dt $ex --steps 3 --warmup 1 --no-extras --parity-windows 4 --settle-seconds 0.1 > $OUT/${tag}_$C.log 2>&1 || { echo "$tag $C failed"; tail -3 $OUT/${tag}_$C.log; exit 1; }
    echo "$tag $C ok"
  done
done
