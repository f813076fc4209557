set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stream.py > gpurun_out/r03o_pytest.log 2>&1 || { tail -40 gpurun_out/r03o_pytest.log; exit 1; }
tail -3 gpurun_out/r03o_pytest.log
timeout -k 10 120 python tools/stream_latency.py --frames 64 --out gpurun_out/r03o_stream_latency.json > gpurun_out/r03o_stream_latency.txt 2>&1
cat gpurun_out/r03o_stream_latency.txt | tail -14
timeout -k 10 300 python bench.py --stream --steps 4096 --warmup 128 --cpu-seconds 0 > gpurun_out/r03o_bench_stream.log 2>&1
grep -o '"value": [0-9.]*\|"avg_step_us": [0-9.]*\|"serve_latency_us": {[^}]*}\|"eager_step_latency_us": [0-9.]*\|"parity": {[^}]*}' gpurun_out/r03o_bench_stream.log
