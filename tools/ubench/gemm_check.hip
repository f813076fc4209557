// Conv-GEMM kernel check + timing harness (tool, not product).
//
//   gemm_check <kernel: tp|big|h16> M N K [dil taps residual]
//
// Runs one of the library's conv-GEMM launchers on random 16-bit data and compares
// it with a naive f32 reference kernel (same bf16 inputs, f32 accumulate): prints
// the max error and the first mismatches, then times 10 launches.
// Build: see tools/ubench/build_gemm_check.sh (links the library's objects).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernels.h"

using namespace vp3d;
typedef __bf16 bf16;

__global__ void ref_kernel(const bf16* A, const bf16* W, const float* sc, const float* sh, const bf16* R,
                           float* Y, ConvGemmParams p) {
    const int m = blockIdx.x, n = threadIdx.x + blockIdx.y * blockDim.x;
    if (m >= p.M || n >= p.N) return;
    const int b = m / p.T_out, t = m % p.T_out;
    const int src = b * p.T_in + t * p.stride;
    float acc = 0.f;
    for (int k = 0; k < p.K; ++k) {
        const int tap = k / p.Ktap, c = k % p.Ktap;
        acc += (float)A[(long)(src + tap * p.dil) * p.lda + c] * (float)W[(long)n * p.Kp + k];
    }
    float v = acc * sc[n] + sh[n];
    if (p.relu) v = v > 0.f ? v : 0.f;
    if (R) v += (float)R[(long)(b * p.R_T + t * p.R_stride + p.R_off) * p.ldr + n];
    Y[(long)m * p.ldy + n] = v;
}

static float frand(unsigned& s) {
    s = s * 1664525u + 1013904223u;
    return ((s >> 8) & 0xFFFF) / 32768.0f - 1.0f;
}

int main(int argc, char** argv) {
    if (argc < 5) {
        printf("usage: gemm_check tp|big|h16 M N Cin [dil taps residual]\n");
        return 2;
    }
    const char* kern = argv[1];
    const int M = atoi(argv[2]), N = atoi(argv[3]), Cin = atoi(argv[4]);
    const int dil = argc > 5 ? atoi(argv[5]) : 1;
    const int taps = argc > 6 ? atoi(argv[6]) : 3;
    const int use_r = argc > 7 ? atoi(argv[7]) : 0;
    // one sequence of T_in rows, output T_out = M rows (dilated conv, stride 1)
    const int T_out = M, T_in = M + (taps - 1) * dil;
    const int K = taps * Cin, Kp = K;
    ConvGemmParams p{};
    p.M = M; p.N = N; p.K = K; p.Kp = Kp; p.T_out = T_out; p.T_in = T_in; p.stride = 1; p.dil = dil;
    p.Ktap = Cin; p.lda = Cin; p.relu = 1; p.ldy = N;
    p.R_T = T_in; p.R_stride = 1; p.R_off = (taps - 1) * dil / 2; p.ldr = N;

    unsigned s = 12345;
    std::vector<bf16> hA((size_t)T_in * Cin), hW((size_t)N * Kp), hR((size_t)T_in * N);
    std::vector<float> hsc(N), hsh(N);
    for (auto& v : hA) v = (bf16)frand(s);
    for (auto& v : hW) v = (bf16)(frand(s) * 0.05f);
    for (auto& v : hR) v = (bf16)frand(s);
    for (int n = 0; n < N; ++n) { hsc[n] = 1.0f + 0.5f * frand(s); hsh[n] = 0.1f * frand(s); }
    bf16 *A, *W, *R, *Y;
    float *sc, *sh, *Yr;
    hipMalloc(&A, hA.size() * 2); hipMalloc(&W, hW.size() * 2); hipMalloc(&R, hR.size() * 2);
    hipMalloc(&Y, (size_t)M * N * 2); hipMalloc(&Yr, (size_t)M * N * 4);
    hipMalloc(&sc, N * 4); hipMalloc(&sh, N * 4);
    hipMemcpy(A, hA.data(), hA.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(W, hW.data(), hW.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(R, hR.data(), hR.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(sc, hsc.data(), N * 4, hipMemcpyHostToDevice);
    hipMemcpy(sh, hsh.data(), N * 4, hipMemcpyHostToDevice);
    hipMemset(Y, 0, (size_t)M * N * 2);
    p.A = A; p.W = W; p.scale = sc; p.shift = sh; p.R = use_r ? R : nullptr; p.Y = Y;

    auto launch = [&]() -> hipError_t {
        if (!strcmp(kern, "tp")) return launch_conv_gemm_tp(p, Act::BF16, 0);
        if (!strcmp(kern, "big")) return launch_conv_gemm_big(p, Act::BF16, Act::BF16, 0);
        if (!strcmp(kern, "8p")) return launch_conv_gemm_8p(p, Act::BF16, 0);
        if (!strcmp(kern, "persist")) return launch_conv_gemm_persist(p, Act::BF16, Act::BF16, 0);
        return launch_conv_gemm(p, Act::BF16, Act::BF16, Act::BF16, 0);
    };
    hipError_t e = launch();
    if (e != hipSuccess) { printf("launch failed: %s\n", hipGetErrorString(e)); return 1; }
    hipLaunchKernelGGL(ref_kernel, dim3(M, (N + 255) / 256), dim3(256), 0, 0, A, W, sc, sh,
                       use_r ? R : nullptr, Yr, p);
    hipDeviceSynchronize();
    std::vector<bf16> hY((size_t)M * N);
    std::vector<float> hYr((size_t)M * N);
    hipMemcpy(hY.data(), Y, hY.size() * 2, hipMemcpyDeviceToHost);
    hipMemcpy(hYr.data(), Yr, hYr.size() * 4, hipMemcpyDeviceToHost);
    double maxe = 0;
    long bad = 0;
    for (long i = 0; i < (long)M * N; ++i) {
        const double d = fabs((double)(float)hY[i] - hYr[i]);
        const double tol = 0.02 + 0.01 * fabs(hYr[i]);
        if (d > maxe) maxe = d;
        if (d > tol) {
            if (bad < 12) {
                printf("  mismatch m=%ld n=%ld got %.5f want %.5f", i / N, i % N, (float)hY[i], hYr[i]);
                // where does the value we got live in the reference? (same tile)
                const long m0 = (i / N) / 256 * 256, n0 = (i % N) / 256 * 256;
                int shown = 0;
                for (long mm = m0; mm < m0 + 256 && mm < M && shown < 3; ++mm)
                    for (long nn = n0; nn < n0 + 256 && nn < N && shown < 3; ++nn)
                        if (fabs(hYr[mm * N + nn] - (float)hY[i]) < 2e-3 && fabs(hYr[mm * N + nn]) > 1e-3) {
                            printf("  ~ref(%ld,%ld)", mm, nn);
                            ++shown;
                        }
                printf("\n");
            }
            ++bad;
        }
    }
    printf("%s M=%d N=%d K=%d dil=%d res=%d: max|d|=%.4g  bad=%ld of %ld\n", kern, M, N, K, dil, use_r, maxe,
           bad, (long)M * N);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) launch();
    hipEventRecord(a, 0);
    for (int i = 0; i < 10; ++i) launch();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= 10;
    printf("%s: %.4f ms  %.1f TFLOP/s\n", kern, ms, 2.0 * M * N * K / (ms * 1e-3) / 1e12);
    return bad ? 1 : 0;
}
