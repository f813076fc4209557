// One split-fp16 (f16x3) GEMM layer through the library's own kernels on real operands
// (measurement, not product code): A (M x K) and W (N x K) f32 rows from tools/real_operands.py
// are split on the host as the library splits them (W scaled by 2^e, hi = f16(x), lo =
// f16(x - hi), 32-wide K groups [hi | lo]), run through conv_gemm_q64's and conv_gemm_a4's X3
// modes as a plain GEMM (one tap of K channels), and compared with the exact sums (float64).
//
//   x3_layer_check A.bin W.bin M N K
//
// Per kernel and epilogue form it prints the sign-correlated relative bias
// sum((D - E) sign(E)) / sum(|E|), the least-squares scale eps = sum((D - E) E) / sum(E^2) and
// the relative rms, in units of 2^-24:
//   f32 out, no ReLU      : D = the accumulator x 2^-e (X3 = 2, scale 2^-e, shift 0)
//   f32 out, ReLU         : D = relu(acc 2^-e), E = relu(exact)
//   split out, ReLU       : D = hi + lo of the split output rows (X3 = 1), E = relu(exact)
//   split vs f32 (ReLU)   : the split output against the f32 output of the same kernel
// Build: tools/ubench/build_x3_layer_check.sh (links the library's GEMM objects).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "host.h"
#include "kernels.h"

using namespace vp3d;
using namespace vp3d::host;

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

static std::vector<float> read_f32(const char* path, size_t n) {
    std::vector<float> v(n);
    FILE* f = fopen(path, "rb");
    if (!f || fread(v.data(), 4, n, f) != n) {
        fprintf(stderr, "cannot read %zu floats from %s\n", n, path);
        exit(1);
    }
    fclose(f);
    return v;
}

static void split_rows(const std::vector<float>& x, int rows, int K, std::vector<uint16_t>& out) {
    out.assign((size_t)rows * 2 * K, 0);
    for (int r = 0; r < rows; ++r)
        for (int k = 0; k < K; ++k) {
            const float v = x[(size_t)r * K + k];
            const uint16_t hi = f32_to_f16_rne(v);
            const size_t q = (size_t)r * 2 * K + x3_pos(k);
            out[q] = hi;
            out[q + 32] = f32_to_f16_rne(v - f16_to_f32(hi));
        }
}

struct Stats {
    double sb = 0, sa = 0, se = 0, see = 0, s2 = 0;
    void add(double d, double e) {
        sb += d * (e > 0 ? 1 : e < 0 ? -1 : 0);
        sa += std::fabs(e);
        se += d * e;
        see += e * e;
        s2 += d * d;
    }
    void print(const char* what) const {
        printf("%-34s bias %+8.4f  eps %+8.4f  rms %8.4f  (x 2^-24)\n", what, sb / sa * 0x1p24, se / see * 0x1p24,
               std::sqrt(s2 / see) * 0x1p24);
    }
};

int main(int argc, char** argv) {
    if (argc < 6) {
        printf("usage: x3_layer_check A.bin W.bin M N K\n");
        return 2;
    }
    const int M = atoi(argv[3]), N = atoi(argv[4]), K = atoi(argv[5]);
    if (K % 64 || N % 256 || M % 256) {
        printf("need K %% 64 == 0, N %% 256 == 0, M %% 256 == 0\n");
        return 2;
    }
    std::vector<float> a = read_f32(argv[1], (size_t)M * K), w = read_f32(argv[2], (size_t)N * K);
    float wmax = 0.f;
    for (float v : w) wmax = std::max(wmax, std::fabs(v));
    const int e = 14 - (int)std::floor(std::log2((double)wmax));
    std::vector<float> ws(w.size());
    for (size_t i = 0; i < w.size(); ++i) ws[i] = std::ldexp(w[i], e);
    std::vector<uint16_t> ax, wx;
    split_rows(a, M, K, ax);
    split_rows(ws, N, K, wx);
    // exact sums of the f32 operands (unscaled weights)
    std::vector<double> ex((size_t)M * N);
    for (int m = 0; m < M; ++m)
        for (int n = 0; n < N; ++n) {
            double s = 0;
            const float* ar = &a[(size_t)m * K];
            const float* wr = &w[(size_t)n * K];
            for (int k = 0; k < K; ++k) s += (double)ar[k] * (double)wr[k];
            ex[(size_t)m * N + n] = s;
        }
    uint16_t *dA, *dW, *dY16;
    float *dY32, *dsc, *dsh;
    CHECK(hipMalloc(&dA, ax.size() * 2));
    CHECK(hipMalloc(&dW, wx.size() * 2));
    CHECK(hipMalloc(&dY16, (size_t)M * 2 * N * 2));
    CHECK(hipMalloc(&dY32, (size_t)M * N * 4));
    CHECK(hipMalloc(&dsc, N * 4));
    CHECK(hipMalloc(&dsh, N * 4));
    CHECK(hipMemcpy(dA, ax.data(), ax.size() * 2, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dW, wx.data(), wx.size() * 2, hipMemcpyHostToDevice));
    std::vector<float> sc(N, std::ldexp(1.0f, -e)), sh(N, 0.f);
    CHECK(hipMemcpy(dsc, sc.data(), N * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dsh, sh.data(), N * 4, hipMemcpyHostToDevice));
    printf("M=%d N=%d K=%d e=%d outputs=%d (units: 2^-24 relative)\n", M, N, K, e, M * N);

    ConvGemmParams p{};
    p.A = dA;
    p.W = dW;
    p.scale = dsc;
    p.shift = dsh;
    p.R = nullptr;
    p.M = M;
    p.N = N;
    p.K = K;
    p.Kp = 2 * K;
    p.T_out = M;
    p.T_in = M;
    p.stride = 1;
    p.dil = 1;
    p.Ktap = 2 * K;
    p.lda = 2 * K;
    p.ldr = 2 * N;
    for (int kern = 0; kern < 2; ++kern) {
        const char* kn = kern == 0 ? "q64" : "a4";
        auto run = [&](bool out_f32, int relu) {
            ConvGemmParams q = p;
            q.relu = relu;
            q.Y = out_f32 ? (void*)dY32 : (void*)dY16;
            q.ldy = out_f32 ? N : 2 * N;
            CHECK(kern == 0 ? launch_conv_gemm_q64_x3(q, out_f32, 0) : launch_conv_gemm_a4_x3(q, out_f32, 0));
            CHECK(hipDeviceSynchronize());
        };
        std::vector<float> y32((size_t)M * N), y32r((size_t)M * N);
        std::vector<uint16_t> y16((size_t)M * 2 * N);
        run(true, 0);
        CHECK(hipMemcpy(y32.data(), dY32, y32.size() * 4, hipMemcpyDeviceToHost));
        run(true, 1);
        CHECK(hipMemcpy(y32r.data(), dY32, y32r.size() * 4, hipMemcpyDeviceToHost));
        run(false, 1);
        CHECK(hipMemcpy(y16.data(), dY16, y16.size() * 2, hipMemcpyDeviceToHost));
        Stats raw, relu32, relu16, s_vs_f;
        for (int m = 0; m < M; ++m)
            for (int n = 0; n < N; ++n) {
                const size_t i = (size_t)m * N + n;
                const double E = ex[i], Er = E > 0 ? E : 0.0;
                raw.add((double)y32[i] - E, E);
                relu32.add((double)y32r[i] - Er, Er);
                const size_t q = (size_t)m * 2 * N + x3_pos(n);
                const double hl = (double)f16_to_f32(y16[q]) + (double)f16_to_f32(y16[q + 32]);
                relu16.add(hl - Er, Er);
                s_vs_f.add(hl - (double)y32r[i], (double)y32r[i]);
            }
        char t[64];
        snprintf(t, sizeof t, "%s f32 out, no ReLU", kn);
        raw.print(t);
        snprintf(t, sizeof t, "%s f32 out, ReLU", kn);
        relu32.print(t);
        snprintf(t, sizeof t, "%s split out, ReLU", kn);
        relu16.print(t);
        snprintf(t, sizeof t, "%s split vs f32 (ReLU)", kn);
        s_vs_f.print(t);
    }
    return 0;
}
