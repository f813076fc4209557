#!/bin/bash
# Build the conv-GEMM check harness: the library's GEMM objects, with the 8p kernel
# recompiled under -DVP3D_ABLATION so VP3D_ABL=1..4,7 select the ablated main loops
# (and the q64 kernel, where VP3D_ABL=1 drops the output traffic, 2 the epilogue; the a4
# kernel, where VP3D_ABL=1 drops the loop DMA, 2 the loop fragment reads, 3 both)
# (measurement only; the product library never contains them).
set -e
cd "$(dirname "$0")"
B=../../dynamic-camera-augmented-videopose3d_amd/build
CS=../../dynamic-camera-augmented-videopose3d_amd/csrc
FL="-x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I ../../include -I $CS -Wno-unused-result -Wno-unused-value"
hipcc $FL -c gemm_check.hip -o /tmp/gemm_check.o
hipcc $FL -DVP3D_ABLATION -c $CS/conv_gemm_8p.hip -o /tmp/conv_gemm_8p_abl.o
hipcc $FL -DVP3D_ABLATION -c $CS/conv_gemm_q64.hip -o /tmp/conv_gemm_q64_abl.o
hipcc $FL -DVP3D_ABLATION -c $CS/conv_gemm_a4.hip -o /tmp/conv_gemm_a4_abl.o
hipcc --offload-arch=gfx950 -o gemm_check /tmp/gemm_check.o $B/conv_gemm.hip.o $B/conv_gemm_big.hip.o /tmp/conv_gemm_a4_abl.o \
  /tmp/conv_gemm_q64_abl.o /tmp/conv_gemm_8p_abl.o
