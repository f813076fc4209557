set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/stream_latency.py --frames 64 --out gpurun_out/r03n_stream_latency.json > gpurun_out/r03n_stream_latency.txt 2>&1
tail -14 gpurun_out/r03n_stream_latency.txt
