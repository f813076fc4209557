// Sustained bf16 MFMA rate on this device: every wave issues independent
// v_mfma_f32_16x16x32_bf16 or v_mfma_f32_32x32x16_bf16 back to back on random register
// operands (no memory traffic inside the loop), 2 waves per SIMD, all CUs.  Reports
// TFLOP/s and the in-kernel clock (s_memtime / s_memrealtime, 100 MHz).  Measurement
// only: the ceiling the conv-GEMM's roofline fraction is read against (DVFS give-back,
// MI355X_MICROARCH.md).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int SHAPE>
__global__ __launch_bounds__(512) void mfma_loop(int iters, float* out, unsigned long long* clk) {
    bf16x8 a, b;
    unsigned s = threadIdx.x * 2654435761u + blockIdx.x * 40503u;
    for (int i = 0; i < 8; ++i) {
        s = s * 1664525u + 1013904223u;
        a[i] = (__bf16)((float)(s >> 8) * 5.96e-8f - 0.5f);
        s = s * 1664525u + 1013904223u;
        b[i] = (__bf16)((float)(s >> 8) * 5.96e-8f - 0.5f);
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float acc_out = 0.f;
    if constexpr (SHAPE == 16) {
        f32x4 c[8];
        for (int j = 0; j < 8; ++j) c[j] = f32x4{0, 0, 0, 0};
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int j = 0; j < 8; ++j) c[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c[j], 0, 0, 0);
        for (int j = 0; j < 8; ++j) acc_out += c[j][0] + c[j][3];
    } else {
        f32x16 c[4];
        for (int j = 0; j < 4; ++j)
            for (int e = 0; e < 16; ++e) c[j][e] = 0.f;
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int j = 0; j < 4; ++j) c[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c[j], 0, 0, 0);
        for (int j = 0; j < 4; ++j) acc_out += c[j][0] + c[j][15];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc_out;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 1;  // 512 threads = 8 waves per CU = 2 per SIMD
    float* out;
    unsigned long long* clk;
    hipMalloc(&out, (size_t)blocks * 512 * 4);
    hipMalloc(&clk, (size_t)blocks * 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 20000;
    for (int shape : {16, 32}) {
        for (int rep = 0; rep < 6; ++rep) {
            hipEventRecord(e0);
            if (shape == 16)
                hipLaunchKernelGGL(mfma_loop<16>, dim3(blocks), dim3(512), 0, 0, iters, out, clk);
            else
                hipLaunchKernelGGL(mfma_loop<32>, dim3(blocks), dim3(512), 0, 0, iters, out, clk);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            // FLOP per MFMA: 16x16x32 -> 16384, 32x32x16 -> 32768; 8 resp. 4 per iteration
            const double flop = (double)blocks * 8 * iters * (shape == 16 ? 8.0 * 16384 : 4.0 * 32768);
            unsigned long long h[2];
            hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
            printf("shape %dx%d: %.3f ms  %.1f TFLOP/s  clock %.2f GHz (block 0)\n", shape, shape, ms,
                   flop / (ms * 1e-3) / 1e12, (double)h[0] / (double)h[1] * 0.1);
        }
    }
    return 0;
}
