#!/bin/bash
# Build the f16x3 1x1 + residual timing harness against an ablation build of conv_gemm_a4.hip.
set -e
cd "$(dirname "$0")"
CS=../../dynamic-camera-augmented-videopose3d_amd/csrc
FL="-x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I ../../include -I $CS -Wno-unused-result -Wno-unused-value"
hipcc $FL -c x3_1x1_check.hip -o /tmp/x3_1x1_check.o
hipcc $FL -DVP3D_ABLATION -c $CS/conv_gemm_a4.hip -o /tmp/conv_gemm_a4_abl.o
hipcc --offload-arch=gfx950 -o x3_1x1_check /tmp/x3_1x1_check.o /tmp/conv_gemm_a4_abl.o
