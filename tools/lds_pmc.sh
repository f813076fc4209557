set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lds
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/lds/avail.txt 2>&1 || true
BENCH_ARGS="--dtype bf16 --no-extras --no-legs" bash tools/pmc_pass.sh lds/bf16 "GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS" && \
BENCH_ARGS="--dtype f16x3 --no-extras --no-legs" bash tools/pmc_pass.sh lds/f16x3 "GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS"
