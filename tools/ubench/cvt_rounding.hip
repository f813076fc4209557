// Rounding of the f32 -> f16 / bf16 conversions the kernels use on gfx950 (measurement, not
// product code): scalar (_Float16)x (v_cvt_f16_f32) and the packed two-value conversion
// (__builtin_convertvector: v_cvt_pk_f16_f32 / v_cvt_pk_bf16_f32), against host
// round-to-nearest-even, over normal, f16-subnormal and halfway inputs.
//   hipcc --offload-arch=gfx950 -O2 -o tools/ubench/cvt_rounding tools/ubench/cvt_rounding.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef __bf16 b2 __attribute__((ext_vector_type(2)));

__global__ void cvt(const float* x, unsigned short* s16, unsigned short* p16, unsigned short* pb16, int n) {
    const int i = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
    if (i + 1 >= n) return;
    const _Float16 a = (_Float16)x[i], b = (_Float16)x[i + 1];
    s16[i] = __builtin_bit_cast(unsigned short, a);
    s16[i + 1] = __builtin_bit_cast(unsigned short, b);
    // the packed instructions themselves, as inline asm: compiled from __builtin_convertvector
    // here (with the scalar conversions of the same pair in view) the compiler emitted
    // v_cvt_pk_f16_f32 v3, v2, v2 / v_cvt_pk_bf16_f32 v2, v2, v2 -- element 0 twice, a
    // miscompile of this test kernel; the library's kernels hold no such operand pair (their
    // ISA was scanned for it)
    unsigned ph, pb;
    asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(ph) : "v"(x[i]), "v"(x[i + 1]));
    asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(pb) : "v"(x[i]), "v"(x[i + 1]));
    const h2 p = __builtin_bit_cast(h2, ph);
    p16[i] = __builtin_bit_cast(unsigned short, p[0]);
    p16[i + 1] = __builtin_bit_cast(unsigned short, p[1]);
    const b2 q = __builtin_bit_cast(b2, pb);
    pb16[i] = __builtin_bit_cast(unsigned short, q[0]);
    pb16[i + 1] = __builtin_bit_cast(unsigned short, q[1]);
}

static unsigned short bf16_rne(float f) {
    unsigned u;
    memcpy(&u, &f, 4);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (unsigned short)(u >> 16);
}

int main() {
    const int n = 1 << 22;
    std::vector<float> x(n);
    unsigned s = 12345;
    for (int i = 0; i < n; ++i) {
        s = s * 1664525u + 1013904223u;
        const int cls = i % 4;
        float v;
        if (cls == 0) v = std::ldexp((float)((s >> 8) & 0xFFFF) / 65536.f + 1.f, (int)((s >> 4) % 20) - 10);  // normal
        else if (cls == 1) v = std::ldexp((float)((s >> 8) & 0xFFFFF) / 1048576.f, -14 - (int)((s >> 3) % 10));  // f16 subnormal range
        else if (cls == 2) {
            // halfway between two f16 values (tie)
            const _Float16 h = (_Float16)std::ldexp(1.f + (float)((s >> 8) & 0x3FF) / 1024.f, (int)((s >> 4) % 10) - 5);
            v = (float)h + std::ldexp(1.f, (int)std::floor(std::log2((float)h)) - 11);
        } else v = std::ldexp((float)((s >> 8) & 0xFFFFFF) / 16777216.f + 1.f, (int)((s >> 4) % 10) - 5);
        if (s & 1) v = -v;
        x[i] = v;
    }
    float* dx;
    unsigned short *ds, *dp, *db;
    hipMalloc(&dx, n * 4);
    hipMalloc(&ds, n * 2);
    hipMalloc(&dp, n * 2);
    hipMalloc(&db, n * 2);
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(cvt, dim3(n / 512), dim3(256), 0, 0, dx, ds, dp, db, n);
    std::vector<unsigned short> hs(n), hp(n), hb(n);
    hipMemcpy(hs.data(), ds, n * 2, hipMemcpyDeviceToHost);
    hipMemcpy(hp.data(), dp, n * 2, hipMemcpyDeviceToHost);
    hipMemcpy(hb.data(), db, n * 2, hipMemcpyDeviceToHost);
    const char* cls_name[4] = {"normal", "f16-subnormal", "f16 tie", "normal 24-bit"};
    long bad_s[4] = {0}, bad_p[4] = {0}, bad_b[4] = {0}, tot[4] = {0};
    double dir_s[4] = {0}, dir_p[4] = {0};
    for (int i = 0; i < n; ++i) {
        const int c = i % 4;
        const _Float16 r = (_Float16)x[i];  // host: round to nearest even (compiler-rt / F16C)
        unsigned short ru;
        memcpy(&ru, &r, 2);
        ++tot[c];
        _Float16 gs, gp;
        memcpy(&gs, &hs[i], 2);
        memcpy(&gp, &hp[i], 2);
        if (hs[i] != ru) {
            ++bad_s[c];
            dir_s[c] += (std::fabs((double)gs) < std::fabs((double)r)) ? -1 : 1;
        }
        if (hp[i] != ru) {
            ++bad_p[c];
            dir_p[c] += (std::fabs((double)gp) < std::fabs((double)r)) ? -1 : 1;
        }
        if (hb[i] != bf16_rne(x[i])) ++bad_b[c];
    }
    for (int c = 0; c < 4; ++c)
        printf("%-14s n=%ld  scalar f16 != RNE: %ld (toward zero %+.0f)  packed f16 != RNE: %ld (toward zero %+.0f)  "
               "packed bf16 != RNE: %ld\n",
               cls_name[c], tot[c], bad_s[c], -dir_s[c], bad_p[c], -dir_p[c], bad_b[c]);
    return 0;
}
