#!/bin/bash
# Build the split-fp16 layer check (tools/ubench/x3_layer_check.hip) against the library's
# GEMM objects (build libvp3d.so first: vp3d_amd/build.py leaves the objects in build/).
set -e
cd "$(dirname "$0")"
B=../../dynamic-camera-augmented-videopose3d_amd/build
CS=../../dynamic-camera-augmented-videopose3d_amd/csrc
FL="-x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I ../../include -I $CS -Wno-unused-result -Wno-unused-value"
hipcc $FL -c x3_layer_check.hip -o /tmp/x3_layer_check.o
hipcc --offload-arch=gfx950 -o x3_layer_check /tmp/x3_layer_check.o $B/conv_gemm.hip.o $B/conv_gemm_big.hip.o $B/conv_gemm_8p.hip.o $B/conv_gemm_a4.hip.o $B/conv_gemm_q64.hip.o
