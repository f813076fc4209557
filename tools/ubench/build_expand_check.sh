#!/bin/bash
# Build the expand-conv harness against an ablation build of expand_gemm.hip.
set -e
cd "$(dirname "$0")"
CS=../../dynamic-camera-augmented-videopose3d_amd/csrc
FL="-x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I ../../include -I $CS -Wno-unused-result"
hipcc $FL -c expand_check.hip -o /tmp/expand_check.o
hipcc $FL -DVP3D_ABLATION -c $CS/expand_gemm.hip -o /tmp/expand_gemm_abl.o
hipcc --offload-arch=gfx950 -o expand_check /tmp/expand_check.o /tmp/expand_gemm_abl.o
