set -o pipefail
mkdir -p gpurun_out/r03j
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stream.py > gpurun_out/r03j/pytest.log 2>&1 || { tail -40 gpurun_out/r03j/pytest.log; exit 1; }
tail -1 gpurun_out/r03j/pytest.log
run() {
  local name=$1; shift
  env "$@" timeout -k 10 120 python tools/stream_latency.py --frames 64 --out gpurun_out/r03j/$name.json > gpurun_out/r03j/$name.txt 2>&1 || { tail -5 gpurun_out/r03j/$name.txt; exit 1; }
  echo "== $name $*"; grep -E "k2 |p2 |host wall" gpurun_out/r03j/$name.txt
}
run base VP3D_STREAM_POLL_ROUNDS=1
run r2 VP3D_STREAM_POLL_ROUNDS=2
run pause8 VP3D_STREAM_POLL_PAUSE=8
run pause32 VP3D_STREAM_POLL_PAUSE=32
run stride512 VP3D_STREAM_CHUNK_STRIDE=512
run stride512r2 VP3D_STREAM_CHUNK_STRIDE=512 VP3D_STREAM_POLL_ROUNDS=2
run pause0 VP3D_STREAM_POLL_PAUSE=0
run contig VP3D_STREAM_ROWS=contig
run contig_r2 VP3D_STREAM_ROWS=contig VP3D_STREAM_POLL_ROUNDS=2
VP3D_STREAM_ROWS=contig timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stream.py > gpurun_out/r03j/pytest_contig.log 2>&1 || { tail -40 gpurun_out/r03j/pytest_contig.log; exit 1; }
tail -1 gpurun_out/r03j/pytest_contig.log
