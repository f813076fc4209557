// Numerical behaviour of v_mfma_f32_16x16x32_f16 on gfx950 (measurement, not product
// code): how the 32 exact f16 products of one output are combined with the f32
// accumulator C.  Each probe fills every lane's A / B fragment with the same pattern
// (so every D element sees the same 32 products) and prints D[0] against the exact sum.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/ubench/mfma_rounding tools/ubench/mfma_rounding.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// a[k], b[k] for k = 0..31 (the K dimension); lane l supplies k = 8 (l >> 4) + 0..7
__global__ void probe(const _Float16* a, const _Float16* b, float c, float* out) {
    const int lane = threadIdx.x;
    f16x8 av, bv;
    for (int e = 0; e < 8; ++e) {
        av[e] = a[8 * (lane >> 4) + e];
        bv[e] = b[8 * (lane >> 4) + e];
    }
    f32x4 acc = {c, c, c, c};
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
    out[lane] = acc[0];
}

static float run(const std::vector<float>& a, const std::vector<float>& b, float c) {
    std::vector<_Float16> ha(32), hb(32);
    for (int k = 0; k < 32; ++k) {
        ha[k] = (_Float16)a[k];
        hb[k] = (_Float16)b[k];
    }
    _Float16 *da, *db;
    float* dout;
    hipMalloc(&da, 64);
    hipMalloc(&db, 64);
    hipMalloc(&dout, 64 * 4);
    hipMemcpy(da, ha.data(), 64, hipMemcpyHostToDevice);
    hipMemcpy(db, hb.data(), 64, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, c, dout);
    float out[64];
    hipMemcpy(out, dout, 64 * 4, hipMemcpyDeviceToHost);
    hipFree(da);
    hipFree(db);
    hipFree(dout);
    return out[0];
}

static void report(const char* what, const std::vector<float>& a, const std::vector<float>& b, float c) {
    double exact = c;
    for (int k = 0; k < 32; ++k) exact += (double)(_Float16)a[k] * (double)(_Float16)b[k];
    const float d = run(a, b, c);
    const float rne = (float)exact;
    const float rz = (float)std::trunc(exact * 0x1p23 / std::pow(2.0, std::floor(std::log2(std::fabs(exact))))) *
                     (float)std::pow(2.0, std::floor(std::log2(std::fabs(exact)))) / 0x1p23f;
    printf("%-58s D=%.10e  exact=%.10e  RNE(exact)=%.10e  RZ(exact)=%.10e  D-exact=%+.3e ulp\n", what, d,
           exact, rne, rz, (d - exact) / (std::pow(2.0, std::floor(std::log2(std::fabs(exact)))) * 0x1p-23));
}

int main() {
    std::vector<float> a(32, 0.f), b(32, 0.f);
    const float u = 0x1p-23f;  // ulp of 1.0
    // 1) one product of +0.75 ulp onto C = 1: RNE -> 1 + ulp, RZ -> 1
    a[0] = 0.75f * u * 0x1p12f;  b[0] = 0x1p-12f;
    report("C=1, +0.75ulp", a, b, 1.0f);
    // 2) -0.75 ulp(1-) onto C = 1: RNE -> 1 - 2^-24 (next below), RZ -> 1 - 2^-24
    a[0] = -0.75f * u * 0x1p12f;
    report("C=1, -0.75ulp", a, b, 1.0f);
    // 3) +0.25 ulp: RNE and RZ -> 1; RU -> 1 + ulp
    a[0] = 0.25f * u * 0x1p12f;
    report("C=1, +0.25ulp", a, b, 1.0f);
    // 4) 32 products of 2^-28 (sum = 1 ulp): summed first -> 1 + ulp; sequential RNE -> 1
    for (int k = 0; k < 32; ++k) { a[k] = 0x1p-14f; b[k] = 0x1p-14f; }
    report("C=1, 32 x 2^-28 (sum 1 ulp)", a, b, 1.0f);
    // 5) 32 products of 2^-30 (sum 0.25 ulp)
    for (int k = 0; k < 32; ++k) { a[k] = 0x1p-15f; b[k] = 0x1p-15f; }
    report("C=1, 32 x 2^-30 (sum 0.25 ulp)", a, b, 1.0f);
    // 6) 16 x +2^-26 and 16 x 2^-26 (sum 32 x 2^-26 = 0.5 ulp): tie -> RNE even (1)
    for (int k = 0; k < 32; ++k) { a[k] = 0x1p-13f; b[k] = 0x1p-13f; }
    report("C=1, 32 x 2^-26 (sum 0.5 ulp, tie)", a, b, 1.0f);
    // 7) large cancellation: 1 + 2^-11 - 1 products with C = 2^-20
    for (int k = 0; k < 32; ++k) { a[k] = 0.f; b[k] = 0.f; }
    a[0] = 1.0f; b[0] = 1.0f + 0x1p-10f; a[1] = -1.0f; b[1] = 1.0f;
    report("C=2^-20, 1*(1+2^-10) - 1*1", a, b, 0x1p-20f);
    // 8) subnormal f16 operands: 2^-20 * 2^-4 onto C = 0
    for (int k = 0; k < 32; ++k) { a[k] = 0.f; b[k] = 0.f; }
    a[0] = 0x1p-20f; b[0] = 0x1p-4f;
    report("C=0, subnormal a=2^-20 times 2^-4", a, b, 0.0f);
    // 9) random mix vs exact, 2000 trials: mean signed error in ulps of |D|
    double bias = 0, rms = 0;
    unsigned s = 12345;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xFFFF) / 32768.0f - 1.0f; };
    const int trials = 2000;
    for (int t = 0; t < trials; ++t) {
        for (int k = 0; k < 32; ++k) { a[k] = rnd() * 4; b[k] = rnd() * 0.01f; }
        const float c = rnd() * 50;
        double exact = c;
        for (int k = 0; k < 32; ++k) exact += (double)(_Float16)a[k] * (double)(_Float16)b[k];
        const double d = run(a, b, c);
        const double ulp = std::pow(2.0, std::floor(std::log2(std::fabs(exact)))) * 0x1p-23;
        bias += (d - exact) / ulp * (exact > 0 ? 1 : -1);  // toward +|x| positive
        rms += ((d - exact) / ulp) * ((d - exact) / ulp);
    }
    printf("random: mean signed error toward |exact| %+.3f ulp, rms %.3f ulp over %d trials\n", bias / trials,
           std::sqrt(rms / trials), trials);
    return 0;
}
