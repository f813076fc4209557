set -o pipefail
OUT=gpurun_out/ab1; mkdir -p $OUT
i=0
for E in "VP3D_NONE=1" "VP3D_GEMM=big" "VP3D_GEMM=persist" "VP3D_GEMM=pp" "VP3D_GEMM=tp" "VP3D_GEMM=8p"; do
  i=$((i+1))
  env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/bench_$i.log 2>&1 || exit $?
  echo "[$E] $(python tools/bench_brief.py $OUT/bench_$i.log)" | tee -a $OUT/summary.txt
done
