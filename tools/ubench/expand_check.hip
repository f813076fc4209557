// Expand-conv harness (measurement only): the gathered 16-bit expand kernel of the
// bench (config 4: 243-frame windows of 17-joint sequences, stride 3, K = 102, N = 1024)
// on B windows, checked on sampled rows against a host fp32 sum of the 16-bit operands,
// then timed; with the -DVP3D_ABLATION objects, per ablation (expand_gemm.hip).
//   expand_check B RB [abl...]      (RB 0 = the library's choice)
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kernels.h"

namespace vp3d {
hipError_t expand_gemm_set_ablation(int a);
void expand_gemm_set_rb(int rb);
}
using namespace vp3d;
typedef __hip_bfloat16 bf16;

static float frand(unsigned& s) {
    s = s * 1664525u + 1013904223u;
    return ((s >> 8) & 0xFFFF) / 32768.0f - 1.0f;
}
static float bfr(float x) { return (float)(bf16)x; }

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 65536;
    expand_gemm_set_rb(argc > 2 ? atoi(argv[2]) : 0);
    const int S = 256, L = 2000, F2 = 34, N = 1024, K = 102, KP = 128, TO = 81, LEAD = 121;
    const int M = B * TO;
    unsigned s = 777;
    std::vector<float> kps((size_t)S * L * F2);
    for (auto& v : kps) v = frand(s);
    std::vector<int64_t> off(S);
    std::vector<int32_t> len(S, L), pairs(2 * (size_t)B);
    for (int i = 0; i < S; ++i) off[i] = (int64_t)i * L;
    for (int b = 0; b < B; ++b) {
        pairs[2 * b] = b % S;
        pairs[2 * b + 1] = (int)((s = s * 1664525u + 1013904223u) >> 8) % L;
    }
    std::vector<bf16> w((size_t)N * KP);
    std::vector<float> sc(N), sh(N);
    for (int n = 0; n < N; ++n)
        for (int k = 0; k < KP; ++k) w[(size_t)n * KP + k] = (bf16)(k < K ? frand(s) * 0.2f : 0.f);
    for (int n = 0; n < N; ++n) { sc[n] = 1.f + 0.5f * frand(s); sh[n] = 0.1f * frand(s); }
    // the kernel's weights: BN scale folded in, shift as hi + lo columns at k = K, K + 1
    std::vector<bf16> wf((size_t)N * KP);
    for (int n = 0; n < N; ++n)
        for (int k = 0; k < KP; ++k) {
            float v = 0.f;
            if (k < K) v = (float)w[(size_t)n * KP + k] * sc[n];
            if (k == K) v = sh[n];
            if (k == K + 1) v = sh[n] - bfr(sh[n]);
            wf[(size_t)n * KP + k] = (bf16)v;
        }

    float *d_kps, *d_sc, *d_sh;
    int64_t* d_off;
    int32_t *d_len, *d_pairs;
    bf16 *d_w, *d_y;
    if (hipMalloc(&d_kps, kps.size() * 4) || hipMalloc(&d_sc, N * 4) || hipMalloc(&d_sh, N * 4) ||
        hipMalloc(&d_off, S * 8) || hipMalloc(&d_len, S * 4) || hipMalloc(&d_pairs, pairs.size() * 4) ||
        hipMalloc(&d_w, w.size() * 2) || hipMalloc(&d_y, (size_t)M * N * 2)) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemcpy(d_kps, kps.data(), kps.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_sc, sc.data(), N * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_sh, sh.data(), N * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_off, off.data(), S * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_len, len.data(), S * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_pairs, pairs.data(), pairs.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_w, wf.data(), wf.size() * 2, hipMemcpyHostToDevice);

    ConvGemmParams p{};
    p.M = M; p.N = N; p.K = K; p.Kp = KP; p.Ktap = K; p.lda = F2; p.stride = 3; p.dil = 1;
    p.T_out = TO; p.T_in = 243; p.relu = 1; p.ldy = N;
    p.W = d_w; p.scale = d_sc; p.shift = d_sh; p.Y = d_y;
    GatherSrc g{};
    g.kps = d_kps; g.f2 = F2; g.seq_off = d_off; g.seq_len = d_len; g.pairs = d_pairs; g.lead = LEAD;
    if (!expand_gather_eligible(p, g, Act::BF16, Act::BF16)) { printf("not eligible\n"); return 1; }

    // VP3D_X3=1: the split-fp16 expand (random [hi | lo] weight slabs, timing only)
    const bool x3 = getenv("VP3D_X3") != nullptr;
    if (x3) {
        unsigned short* d_wx;
        unsigned short* d_yx;
        std::vector<unsigned short> wx((size_t)N * 2 * KP);
        for (auto& v : wx) v = (unsigned short)(((s = s * 1664525u + 1013904223u) >> 8) & 0x3BFF);
        if (hipMalloc(&d_wx, wx.size() * 2) || hipMalloc(&d_yx, (size_t)M * N * 4)) { printf("alloc failed\n"); return 1; }
        (void)hipMemcpy(d_wx, wx.data(), wx.size() * 2, hipMemcpyHostToDevice);
        ConvGemmParams q = p;
        q.W = d_wx; q.Kp = 2 * KP; q.ldy = 2 * N; q.Y = d_yx;
        if (!expand_gemm_x3_eligible(q, &g)) { printf("x3 not eligible\n"); return 1; }
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        const int nabl = argc > 3 ? argc - 3 : 1;
        for (int r = 0; r < 3; ++r)
            for (int a = 0; a < nabl; ++a) {
                const int abl = argc > 3 ? atoi(argv[3 + a]) : 0;
                if (expand_gemm_set_ablation(abl) != hipSuccess) { printf("set ablation failed\n"); return 1; }
                for (int i = 0; i < 2; ++i) (void)launch_expand_gemm_x3(q, &g, 0);
                (void)hipEventRecord(e0, 0);
                for (int i = 0; i < 10; ++i) (void)launch_expand_gemm_x3(q, &g, 0);
                (void)hipEventRecord(e1, 0);
                if (hipEventSynchronize(e1) != hipSuccess) { printf("launch failed\n"); return 1; }
                float ms = 0;
                (void)hipEventElapsedTime(&ms, e0, e1);
                ms /= 10;
                printf("x3 round %d abl %d: %.4f ms  %.2f TB/s output\n", r, abl, ms, (double)M * N * 4 / ms / 1e9);
            }
        return 0;
    }
    (void)expand_gemm_set_ablation(0);
    if (launch_expand_gemm_gather(p, g, Act::BF16, 0) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        printf("launch failed\n");
        return 1;
    }
    std::vector<bf16> y((size_t)M * N);
    (void)hipMemcpy(y.data(), d_y, y.size() * 2, hipMemcpyDeviceToHost);
    double maxd = 0;
    int bad = 0;
    for (int q = 0; q < 512; ++q) {
        const int m = (int)(((unsigned long long)q * 2654435761ull) % M);
        const int b = m / TO, t = m % TO;
        const int sq = pairs[2 * b], f0 = pairs[2 * b + 1] - LEAD + 3 * t;
        for (int n = 0; n < N; ++n) {
            float acc = 0.f;
            for (int k = 0; k < K; ++k) {
                int fr = f0 + k / F2;
                fr = fr < 0 ? 0 : (fr >= L ? L - 1 : fr);
                acc += bfr(kps[((size_t)off[sq] + fr) * F2 + k % F2]) * (float)w[(size_t)n * KP + k];
            }
            float r = acc * sc[n] + sh[n];
            r = r > 0.f ? r : 0.f;
            const float got = (float)y[(size_t)m * N + n];
            const double d = fabs(got - r);
            if (d > maxd) maxd = d;
            if (d > 0.02 + 0.01 * fabs(r)) ++bad;
        }
    }
    printf("expand B=%d M=%d RB=%s: max|d|=%.4g bad=%d of %d\n", B, M, argc > 2 ? argv[2] : "0", maxd, bad, 512 * N);

    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int nabl = argc > 3 ? argc - 3 : 1;
    for (int r = 0; r < 3; ++r)
        for (int a = 0; a < nabl; ++a) {
            const int abl = argc > 3 ? atoi(argv[3 + a]) : 0;
            if (expand_gemm_set_ablation(abl) != hipSuccess) { printf("set ablation failed\n"); return 1; }
            for (int i = 0; i < 2; ++i) (void)launch_expand_gemm_gather(p, g, Act::BF16, 0);
            (void)hipEventRecord(e0, 0);
            for (int i = 0; i < 10; ++i) (void)launch_expand_gemm_gather(p, g, Act::BF16, 0);
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            ms /= 10;
            printf("round %d abl %d: %.4f ms  %.2f TB/s output\n", r, abl, ms, (double)M * N * 2 / ms / 1e9);
        }
    return 0;
}
