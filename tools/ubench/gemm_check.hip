// Conv-GEMM kernel check + timing harness (tool, not product).
//
//   gemm_check <kernel: 8p|q64|a4|big|h16> M N K [dil taps residual]
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
#include <algorithm>

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
        printf("usage: gemm_check 8p|q64|a4|big|h16 M N Cin [dil taps residual]\n");
        return 2;
    }
    const char* kern = argv[1];
    const int M = atoi(argv[2]), N = atoi(argv[3]), Cin = atoi(argv[4]);
    const int dil = argc > 5 ? atoi(argv[5]) : 1;
    const int taps = argc > 6 ? atoi(argv[6]) : 3;
    const int use_r = argc > 7 ? atoi(argv[7]) : 0;
    // one sequence of T_in rows, output T_out = M rows (dilated conv, stride 1: output row m
    // reads input rows m + tap * dil, so neighbouring rows share input rows).  VP3D_STRIDE=3
    // with taps 3, dil 1: the Optimized1f strided k3 conv (input rows 3m .. 3m + 2, no sharing:
    // three times the A traffic of stride 1)
    const int stride = getenv("VP3D_STRIDE") ? atoi(getenv("VP3D_STRIDE")) : 1;
    const int T_out = M, T_in = (M - 1) * stride + 1 + (taps - 1) * dil;
    const int K = taps * Cin, Kp = K;
    ConvGemmParams p{};
    p.M = M; p.N = N; p.K = K; p.Kp = Kp; p.T_out = T_out; p.T_in = T_in; p.stride = stride; p.dil = dil;
    p.Ktap = Cin; p.lda = Cin; p.relu = 1; p.ldy = N;
    p.R_T = T_in; p.R_stride = 1; p.R_off = (taps - 1) * dil / 2; p.ldr = N;

    unsigned s = 12345;
    std::vector<bf16> hA((size_t)T_in * Cin), hW((size_t)N * Kp), hR((size_t)T_in * N);
    std::vector<float> hsc(N), hsh(N);
    // VP3D_RELU_A=1: A as a ReLU output (about half zeros, the rest positive), as the lifter's
    // block inputs are
    const bool relu_a = getenv("VP3D_RELU_A") != nullptr;
    for (auto& v : hA) {
        const float x = frand(s);
        v = (bf16)(relu_a ? (x > 0.f ? x : 0.f) : x);
    }
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

    const bool trace = !strcmp(kern, "8pt") || !strcmp(kern, "a4t");
    const bool a4t = !strcmp(kern, "a4t");
    unsigned long long* d_trace = nullptr;
    const int nwg_trace = ((M + 255) / 256) * (N / 256);
    if (trace) {
        // the buffer is in place before the first launch (VP3D_ABL=7 launches write it)
        hipMalloc(&d_trace, (size_t)nwg_trace * 80);
        hipMemset(d_trace, 0, (size_t)nwg_trace * 80);
        if ((a4t ? conv_gemm_a4_set_trace(d_trace) : conv_gemm_8p_set_trace(d_trace)) != hipSuccess) {
            printf("set_trace failed\n");
            return 1;
        }
        // a4t: VP3D_ABL 4 (default), 12 (stores dropped) or 20 (no epilogue) from the environment
        if (a4t) {
            const char* e = getenv("VP3D_ABL");
            if (!e || (atoi(e) & 4) == 0) setenv("VP3D_ABL", "4", 1);
        } else {
            setenv("VP3D_ABL", "7", 1);
        }
        kern = a4t ? "a4" : "8p";
    }
    auto launch = [&]() -> hipError_t {
        if (!strcmp(kern, "big")) return launch_conv_gemm_big(p, Act::BF16, Act::BF16, 0);
        if (!strcmp(kern, "8p")) return launch_conv_gemm_8p(p, Act::BF16, 0);
        if (!strcmp(kern, "q64")) return launch_conv_gemm_q64(p, Act::BF16, 0);
        if (!strcmp(kern, "a4")) return launch_conv_gemm_a4(p, Act::BF16, 0);
        return launch_conv_gemm(p, Act::BF16, Act::BF16, Act::BF16, 0);
    };
    hipError_t e = launch();
    if (e != hipSuccess) { printf("launch failed: %s\n", hipGetErrorString(e)); return 1; }
    // VP3D_NOCHECK=1: no reference comparison (timing / stamps of shapes too large to check)
    double maxe = 0;
    long bad = 0;
    if (!getenv("VP3D_NOCHECK")) {
    hipLaunchKernelGGL(ref_kernel, dim3(M, (N + 255) / 256), dim3(256), 0, 0, A, W, sc, sh,
                       use_r ? R : nullptr, Yr, p);
    hipDeviceSynchronize();
    std::vector<bf16> hY((size_t)M * N);
    std::vector<float> hYr((size_t)M * N);
    hipMemcpy(hY.data(), Y, hY.size() * 2, hipMemcpyDeviceToHost);
    hipMemcpy(hYr.data(), Yr, hYr.size() * 4, hipMemcpyDeviceToHost);
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
    }
    printf("%s M=%d N=%d K=%d dil=%d res=%d: max|d|=%.4g  bad=%ld of %ld\n", kern, M, N, K, dil, use_r, maxe,
           bad, (long)M * N);
    if (trace) {
        // one traced launch: per-workgroup start / prologue done / K loop done / stores
        // retired (100 MHz wall clock), grouped by the CU each workgroup ran on
        const int nwg = nwg_trace;
        unsigned long long* d = d_trace;
        for (int i = 0; i < 3; ++i) launch();
        hipDeviceSynchronize();
        std::vector<unsigned long long> t((size_t)nwg * 10);
        hipMemcpy(t.data(), d, t.size() * 8, hipMemcpyDeviceToHost);
        unsigned long long t0 = ~0ull, t1 = 0;
        for (int w = 0; w < nwg; ++w) { t0 = std::min(t0, t[w * 10]); t1 = std::max(t1, t[w * 10 + 3]); }
        double pro = 0, loop = 0, epi = 0, cpro = 0, cloop = 0, cepi = 0;
        for (int w = 0; w < nwg; ++w) {
            const unsigned long long* r = &t[w * 10];
            pro += r[1] - r[0]; loop += r[2] - r[1]; epi += r[3] - r[2];
            cpro += r[6] - r[5]; cloop += r[7] - r[6]; cepi += r[8] - r[7];
        }
        if (a4t) {
            double mid = 0;
            for (int w = 0; w < nwg; ++w) mid += t[w * 10 + 9];
            printf("trace: wave 0 in the mid waits + barriers %.0f cycles per WG (%.1f %% of the K loop)\n",
                   mid / nwg, 100.0 * mid / cloop);
        }
        printf("trace: kernel span %.1f us; per WG mean: prologue %.2f us, K loop %.2f us, epilogue %.2f us"
               " (cycles %.0f / %.0f / %.0f -> %.2f GHz in loop)\n", (t1 - t0) / 100.0, pro / nwg / 100.0,
               loop / nwg / 100.0, epi / nwg / 100.0, cpro / nwg, cloop / nwg, cepi / nwg,
               cloop / (loop / 100.0) / 1e3);
        // per CU: sorted workgroups, gaps between one's end and the next's start
        std::vector<std::pair<unsigned long long, int>> key;
        for (int w = 0; w < nwg; ++w) key.push_back({(t[w * 10 + 4] & 0xFFFFFFFF0000FF00ull) , w});
        std::sort(key.begin(), key.end(), [&](auto& x, auto& y) {
            return x.first != y.first ? x.first < y.first : t[x.second * 10] < t[y.second * 10]; });
        double gap = 0; long ng = 0; int ncu = 0;
        for (size_t i = 0; i < key.size(); ++i) {
            if (i == 0 || key[i].first != key[i - 1].first) { ++ncu; continue; }
            gap += (double)t[key[i].second * 10] - (double)t[key[i - 1].second * 10 + 3]; ++ng;
        }
        printf("trace: %d distinct CUs, mean gap end->next start on a CU %.2f us (%ld gaps)\n", ncu,
               ng ? gap / ng / 100.0 : 0.0, ng);
        // round-by-round: start times of the i-th workgroup on each CU, relative to t0
        for (int round = 0; round < 16; ++round) {
            double smin = 1e30, smax = 0, emin = 1e30, emax = 0; int cnt = 0;
            size_t i = 0;
            while (i < key.size()) {
                size_t j = i; while (j < key.size() && key[j].first == key[i].first) ++j;
                if (i + round < j) {
                    const unsigned long long* r = &t[key[i + round].second * 10];
                    smin = std::min(smin, (double)(r[0] - t0)); smax = std::max(smax, (double)(r[0] - t0));
                    emin = std::min(emin, (double)(r[3] - t0)); emax = std::max(emax, (double)(r[3] - t0));
                    ++cnt;
                }
                i = j;
            }
            if (!cnt) break;
            printf("  round %2d: %3d WGs start %.1f..%.1f us, end %.1f..%.1f us\n", round, cnt, smin / 100,
                   smax / 100, emin / 100, emax / 100);
        }
        return 0;
    }
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    // VP3D_WARM / VP3D_ITERS: untimed / timed launches (default 3 / 10)
    const int nwarm = getenv("VP3D_WARM") ? atoi(getenv("VP3D_WARM")) : 3;
    const int niter = getenv("VP3D_ITERS") ? atoi(getenv("VP3D_ITERS")) : 10;
    for (int i = 0; i < nwarm; ++i) launch();
    hipEventRecord(a, 0);
    for (int i = 0; i < niter; ++i) launch();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= niter;
    printf("%s: %.4f ms  %.1f TFLOP/s\n", kern, ms, 2.0 * M * N * K / (ms * 1e-3) / 1e12);
    return bad ? 1 : 0;
}
