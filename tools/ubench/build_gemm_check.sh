#!/bin/bash
# Build the conv-GEMM check harness against the library's compiled objects.
set -e
cd "$(dirname "$0")"
B=../../dynamic-camera-augmented-videopose3d_amd/build
hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -I ../../include -I ../../dynamic-camera-augmented-videopose3d_amd/csrc \
  -c gemm_check.hip -o /tmp/gemm_check.o
hipcc --offload-arch=gfx950 -o gemm_check /tmp/gemm_check.o $B/conv_gemm.hip.o $B/conv_gemm_big.hip.o \
  $B/conv_gemm_persist.hip.o $B/conv_gemm_pp.hip.o $B/conv_gemm_tp.hip.o $B/conv_gemm_8p.hip.o $B/conv_gemm_8pp.hip.o
