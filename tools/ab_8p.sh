set -o pipefail
OUT=gpurun_out/ab2; mkdir -p $OUT
cd tools/ubench
for k in 8p big; do timeout -k 5 60 ./gemm_check $k 221184 1024 1024 1 1 1 | tail -2 || exit $?; done > ../../$OUT/gemm.txt
cd ../..
VP3D_GEMM=8p timeout -k 10 300 python -u -m pytest tests/test_gpu_lifter.py tests/test_gpu_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_8p.txt 2>&1 || exit $?
for E in "VP3D_NONE=1" "VP3D_GEMM=8p" "VP3D_NONE=1" "VP3D_GEMM=8p"; do
  i=$((i+1))
  env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/bench_$i.log 2>&1 || exit $?
  echo "[$E] $(python tools/bench_brief.py $OUT/bench_$i.log)" | tee -a $OUT/summary.txt
done
