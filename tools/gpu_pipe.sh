set -o pipefail
mkdir -p gpurun_out/pipe1
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pipe1/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/pipe1/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --stream --steps 4096 --warmup 128 --cpu-seconds 0 > gpurun_out/pipe1/bench_pipe.log 2>&1 || exit $?
tail -1 gpurun_out/pipe1/bench_pipe.log | cut -c1-1500
VP3D_STREAM_MODE=persist timeout -k 10 200 python bench.py --stream --steps 4096 --warmup 128 --cpu-seconds 0 > gpurun_out/pipe1/bench_persist.log 2>&1 || exit $?
tail -1 gpurun_out/pipe1/bench_persist.log | cut -c1-600
