// Timing harness for the split-fp16 (f16x3) conv_gemm_a4 1x1 + residual layer (tool, not
// product): block-1 1x1 of config 4 by default (M = 27 x B rows, N = K = 1024), operands of
// random f16 halves generated on the device, the library's launcher (walked tiles), ablation
// variants from an ablation build of conv_gemm_a4.hip (VP3D_ABL, see a4_x3_abl).
//   x3_1x1_check [B=65536] [abl...]     -> ms per launch, effective TFLOP/s, per ablation
// Build: tools/ubench/build_x3_1x1_check.sh
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>

#include "kernels.h"

using namespace vp3d;

__global__ void fill_f16(unsigned short* p, size_t n, unsigned seed, float scale) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        const float v = ((x & 0xFFFF) / 32768.0f - 1.0f) * scale;
        p[i] = __builtin_bit_cast(unsigned short, (_Float16)v);
    }
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 65536;
    const int M = 27 * B, N = 1024, C = 1024;
    ConvGemmParams p{};
    p.M = M; p.N = N; p.K = C; p.Kp = 2 * C; p.T_out = 27; p.T_in = 81; p.stride = 3; p.dil = 1;
    p.Ktap = 2 * C; p.lda = 2 * C; p.relu = 1; p.ldy = 2 * N;
    p.R_T = 81; p.R_stride = 3; p.R_off = 1; p.ldr = 2 * N;
    // the 1x1 conv reads its own input rows (stride 1 over the k3 output), the residual the
    // block input's rows 3 t + 1 (Optimized1f, TemporalModel.py:192)
    p.T_in = 27; p.stride = 1;
    unsigned short *A, *W, *R, *Y;
    float *sc, *sh;
    const size_t na = (size_t)M * 2 * C, nr = (size_t)B * 81 * 2 * N, ny = (size_t)M * 2 * N;
    if (hipMalloc(&A, na * 2) || hipMalloc(&R, nr * 2) || hipMalloc(&Y, ny * 2) || hipMalloc(&W, (size_t)N * 2 * C * 2) ||
        hipMalloc(&sc, N * 4) || hipMalloc(&sh, N * 4)) {
        printf("alloc failed\n");
        return 1;
    }
    hipLaunchKernelGGL(fill_f16, dim3(4096), dim3(256), 0, 0, A, na, 1u, 1.0f);
    hipLaunchKernelGGL(fill_f16, dim3(4096), dim3(256), 0, 0, R, nr, 2u, 1.0f);
    hipLaunchKernelGGL(fill_f16, dim3(1024), dim3(256), 0, 0, W, (size_t)N * 2 * C, 3u, 0.03f);
    hipLaunchKernelGGL(fill_f16, dim3(8), dim3(256), 0, 0, (unsigned short*)sc, (size_t)N * 2, 4u, 0.5f);
    hipLaunchKernelGGL(fill_f16, dim3(8), dim3(256), 0, 0, (unsigned short*)sh, (size_t)N * 2, 5u, 0.1f);
    hipDeviceSynchronize();
    p.A = A; p.W = W; p.R = R; p.Y = Y; p.scale = sc; p.shift = sh;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int nabl = argc > 2 ? argc - 2 : 1;
    for (int r = 0; r < 2; ++r)
        for (int i = 0; i < nabl; ++i) {
            const std::string abl = argc > 2 ? argv[2 + i] : "0";
            setenv("VP3D_ABL", abl.c_str(), 1);
            // the launcher reads VP3D_ABL once (static): one ablation per process
            if (i > 0 || r > 0) break;
            for (int w = 0; w < 3; ++w) launch_conv_gemm_a4_x3(p, false, 0);
            hipEventRecord(a, 0);
            const int it = 10;
            for (int w = 0; w < it; ++w) launch_conv_gemm_a4_x3(p, false, 0);
            hipEventRecord(b, 0);
            if (hipEventSynchronize(b) != hipSuccess) { printf("launch failed\n"); return 1; }
            float ms;
            hipEventElapsedTime(&ms, a, b);
            ms /= it;
            printf("B=%d abl=%s: %.4f ms  %.1f TFLOP/s (f32-equivalent)\n", B, abl.c_str(), ms,
                   2.0 * M * N * C / (ms * 1e-3) / 1e12);
        }
    return 0;
}
