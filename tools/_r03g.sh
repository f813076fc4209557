set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pipeline.py -k "forward_windows" tests/test_gpu_lifter.py::test_gemm_kernel_override > gpurun_out/r03g_pytest.log 2>&1 || { tail -30 gpurun_out/r03g_pytest.log; exit 1; }
tail -3 gpurun_out/r03g_pytest.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --parity-windows 4 --no-extras > gpurun_out/r03g_q64.log 2>&1
VP3D_GEMM=q4w timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --parity-windows 4 --no-extras > gpurun_out/r03g_q4w.log 2>&1
grep -o '"value": [0-9.]*\|"per_layer_ms": {[^}]*}\|"parity": {[^}]*}' gpurun_out/r03g_q64.log gpurun_out/r03g_q4w.log
timeout -k 10 120 python tools/stream_latency.py --frames 64 --out gpurun_out/r03g_stream_latency.json > gpurun_out/r03g_stream_latency.txt 2>&1
cat gpurun_out/r03g_stream_latency.txt | tail -20
