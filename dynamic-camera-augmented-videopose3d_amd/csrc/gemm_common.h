// Device-side building blocks shared by the conv-GEMM kernel families
// (conv_gemm.hip: 128x128 tiles; conv_gemm_big.hip: 256x256 LDS-DMA tiles).
#pragma once
#include "kernels.h"

// No silent FMA contraction in the epilogues: the BatchNorm affine is applied
// as ATen's CPU kernel applies it (x * alpha, then + beta, two roundings).
#pragma clang fp contract(off)

namespace vp3d {
namespace gemm {

typedef __bf16 bf16;
typedef _Float16 f16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));


__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    // bijective round-robin inverse (cdna_hip_programming.md §5 "XCD swizzle must be bijective")
    const int xcd = bid & 7;
    const int q = nwg >> 3, r = nwg & 7;
    const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (bid >> 3);
}

template <typename T> __device__ __forceinline__ float to_f32(T v) { return (float)v; }

template <typename T> __device__ __forceinline__ T from_f32(float v) { return (T)v; }

template <typename CT> struct Pack8;
template <> struct Pack8<bf16> { typedef bf16x8 type; };
template <> struct Pack8<f16> { typedef f16x8 type; };

template <typename CT>
__device__ __forceinline__ u32x4 pack8(const float (&v)[8]) {
    typename Pack8<CT>::type r;
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = (CT)v[e];
    return __builtin_bit_cast(u32x4, r);
}

template <typename CT>
__device__ __forceinline__ f32x4 mfma16(u32x4 a, u32x4 b, f32x4 c);
template <>
__device__ __forceinline__ f32x4 mfma16<bf16>(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mfma16<f16>(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

__device__ __forceinline__ int src_row(const ConvGemmParams& p, int m) {
    const int b = m / p.T_out;
    const int t = m - b * p.T_out;
    return b * p.T_in + t * p.stride;
}

__device__ __forceinline__ int res_row(const ConvGemmParams& p, int m) {
    const int b = m / p.T_out;
    const int t = m - b * p.T_out;
    return b * p.R_T + t * p.R_stride + p.R_off;
}

// A-operand addressing modes
//   A_SCALAR  general tap mapping, one element at a time (bounds-checked, zero fill)
//   A_PAIRS   one contiguous K segment per row (taps collapsed, dil == 1) of f32
//             activations with an even row pitch: 8-byte loads, no division
//             (the expand conv: K = w0 * J * F = 102 or 138)
//   A_VEC     tap-aligned K tiles (Ktap % BK == 0): 16-byte loads
enum : int { A_SCALAR = 0, A_PAIRS = 1, A_VEC = 2 };

template <typename AT>
__device__ __forceinline__ float load_a_scalar(const ConvGemmParams& p, int srow, int kk) {
    if (kk >= p.K) return 0.f;
    const int tap = kk / p.Ktap;
    const int c = kk - tap * p.Ktap;
    const AT* A = (const AT*)p.A;
    return to_f32(A[(int64_t)(srow + tap * p.dil) * p.lda + c]);
}

// NE consecutive A elements of row `srow` starting at k index kk0 (NE % 2 == 0), as f32.
template <typename AT, int AMODE, int NE>
__device__ __forceinline__ void load_a_run(const ConvGemmParams& p, int srow, int kk0, bool valid,
                                           float (&v)[NE]) {
    if (!valid) {
#pragma unroll
        for (int e = 0; e < NE; ++e) v[e] = 0.f;
        return;
    }
    if constexpr (AMODE == A_PAIRS) {
        const float* row = (const float*)p.A + (int64_t)srow * p.lda;
#pragma unroll
        for (int e = 0; e < NE; e += 2) {
            const int kk = kk0 + e;
            if (kk < p.K) {
                const float2 t = *(const float2*)(row + kk);
                v[e] = t.x;
                v[e + 1] = t.y;
            } else {
                v[e] = v[e + 1] = 0.f;
            }
        }
    } else {
#pragma unroll
        for (int e = 0; e < NE; ++e) v[e] = load_a_scalar<AT>(p, srow, kk0 + e);
    }
}

// ---------------------------------------------------------------------------
// Epilogues
// ---------------------------------------------------------------------------
// Scalar epilogue (any N): straight from the MFMA accumulator layout.
template <typename OT>
__device__ __forceinline__ void epi_store(const ConvGemmParams& p, int m, int n, float v,
                                          float sc, float sh) {
    // BatchNorm eval as ATen's CPU kernel evaluates it: x * alpha + beta, two roundings
    v = __fadd_rn(__fmul_rn(v, sc), sh);
    if (p.relu == 1) v = v > 0.f ? v : 0.f;
    else if (p.relu == 2) v = v > 0.f ? v : v * 0.01f;  // LeakyReLU (nn.LeakyReLU default slope)
    if (p.R) v += to_f32(((const OT*)p.R)[(int64_t)res_row(p, m) * p.ldr + n]);
    ((OT*)p.Y)[(int64_t)m * p.ldy + n] = from_f32<OT>(v);
}

template <typename OT, int MI>
__device__ __forceinline__ void epilogue_scalar(const ConvGemmParams& p, const f32x4 (&acc)[MI][4],
                                                int mw, int nw, int lane) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = nw + j * 16 + (lane & 15);
        if (n >= p.N) continue;
        const float sc = p.scale[n], sh = p.shift[n];
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = mw + i * 16 + (lane >> 4) * 4 + r;
                if (m < p.M) epi_store<OT>(p, m, n, acc[i][j][r], sc, sh);
            }
    }
}

// Vector epilogue (N % 8 == 0): each wave transposes its (16*MI)x64 f32 accumulator
// tile through its own LDS region (row pitch 68 floats: conflict-free writes),
// then every lane owns 8 consecutive columns of a row: 16/32-byte residual loads
// and output stores, whole 128-byte lines per 8 lanes.
//
// No workgroup barrier inside: the staging region is private to the wave and one
// wave's LDS instructions retire in issue order, so a compiler fence orders the
// transpose.  (A __syncthreads here would also wait for every global store issued
// so far, serialising the passes on store completion.)  The residual rows of pass
// k+1 are loaded before the stores of pass k, so waiting for them never waits for
// those stores either.
constexpr int kEpiLd = 68;

template <typename OT, int MI, int PASS_ROWS>
__device__ __forceinline__ void epilogue_vec(const ConvGemmParams& p, const f32x4 (&acc)[MI][4],
                                             float* stage, int mw, int nw, int lane) {
    constexpr int NP = MI * 16 / PASS_ROWS;  // passes
    constexpr int NQ = PASS_ROWS / 8;        // rows per lane per pass
    constexpr int RW = sizeof(OT) == 2 ? 1 : 2;  // 16-byte words per 8 outputs
    const int c8 = lane & 7;
    const int n = nw + c8 * 8;
    const bool nval = n < p.N;
    float sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        sc[e] = nval ? p.scale[n + e] : 0.f;
        sh[e] = nval ? p.shift[n + e] : 0.f;
    }
    u32x4 res[2][NQ][RW];
    auto load_res = [&](int pass, u32x4 (&r)[NQ][RW]) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int m = mw + pass * PASS_ROWS + q * 8 + (lane >> 3);
            if (p.R && m < p.M && nval) {
                const OT* rp = (const OT*)p.R + (int64_t)res_row(p, m) * p.ldr + n;
#pragma unroll
                for (int w = 0; w < RW; ++w) r[q][w] = *(const u32x4*)(rp + w * (16 / sizeof(OT)));
            } else {
#pragma unroll
                for (int w = 0; w < RW; ++w) r[q][w] = u32x4{0u, 0u, 0u, 0u};
            }
        }
    };
    load_res(0, res[0]);
#pragma unroll
    for (int pass = 0; pass < NP; ++pass) {
#pragma unroll
        for (int ii = 0; ii < PASS_ROWS / 16; ++ii) {
            const int i = pass * (PASS_ROWS / 16) + ii;
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    stage[(ii * 16 + (lane >> 4) * 4 + r) * kEpiLd + j * 16 + (lane & 15)] = acc[i][j][r];
        }
        asm volatile("" ::: "memory");
        if (pass + 1 < NP) load_res(pass + 1, res[(pass + 1) & 1]);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int row = q * 8 + (lane >> 3);
            const int m = mw + pass * PASS_ROWS + row;
            const f32x4 lo = *(const f32x4*)&stage[row * kEpiLd + c8 * 8];
            const f32x4 hi = *(const f32x4*)&stage[row * kEpiLd + c8 * 8 + 4];
            if (m < p.M && nval) {
                float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    v[e] = __fadd_rn(__fmul_rn(v[e], sc[e]), sh[e]);
                    if (p.relu == 1) v[e] = v[e] > 0.f ? v[e] : 0.f;
                    else if (p.relu == 2) v[e] = v[e] > 0.f ? v[e] : v[e] * 0.01f;
                }
                if (p.R) {
                    const u32x4(&rq)[RW] = res[pass & 1][q];
                    if constexpr (sizeof(OT) == 2) {
                        typedef OT ot8 __attribute__((ext_vector_type(8)));
                        const ot8 r8 = __builtin_bit_cast(ot8, rq[0]);
#pragma unroll
                        for (int e = 0; e < 8; ++e) v[e] += (float)r8[e];
                    } else {
                        const f32x4 r0 = __builtin_bit_cast(f32x4, rq[0]);
                        const f32x4 r1 = __builtin_bit_cast(f32x4, rq[1]);
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            v[e] += r0[e];
                            v[e + 4] += r1[e];
                        }
                    }
                }
                const int64_t yo = (int64_t)m * p.ldy + n;
                if constexpr (sizeof(OT) == 2) {
                    typedef OT ot8 __attribute__((ext_vector_type(8)));
                    ot8 o;
#pragma unroll
                    for (int e = 0; e < 8; ++e) o[e] = (OT)v[e];
                    *(u32x4*)((OT*)p.Y + yo) = __builtin_bit_cast(u32x4, o);
                } else {
                    *(f32x4*)((float*)p.Y + yo) = f32x4{v[0], v[1], v[2], v[3]};
                    *(f32x4*)((float*)p.Y + yo + 4) = f32x4{v[4], v[5], v[6], v[7]};
                }
            }
        }
        asm volatile("" ::: "memory");
    }
}

// ---------------------------------------------------------------------------
// Register-direct epilogue for the transposed MFMA orientation (D = W . A^T):
// acc[i][j] of a lane holds output channels nw + 16j + 4(lane>>4) + (0..3) of row
// mw + 16i + (lane & 15).  BatchNorm affine + ReLU run in that layout (scale/shift
// from LDS), then one v_permlane16_swap per value pair gives each lane 8
// consecutive channels (nw + 32jp + c0 + 0..7, c0 = 0/16/8/24 for lane>>4 = 0..3),
// the residual is added in f32, converted once, and stored as 16 bytes: every
// store instruction writes 16 rows x 64 B.  Stores (and residual loads) use a
// buffer resource so rows past M are dropped by the range check, not a branch:
// every wave issues exactly 2*MI stores, the count the callers' vmcnt waits use.
// With a residual the loads run one row block ahead of the stores and are waited
// for here (vmcnt(2)/(4): older vector-memory operations are waited for too).
// min(bytes, 2^31 - 1) on scalar ops: a 64-bit compare against the constant becomes a VALU
// v_cmp_lt_u64 whose constant operand the compiler keeps in a VGPR pair for the whole kernel
__device__ __forceinline__ uint32_t clamp_range31(size_t bytes) {
    return (bytes >> 31) != 0 ? 0x7FFFFFFFu : (uint32_t)bytes;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

template <int N>
__device__ __forceinline__ void vm_wait_n() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Residual rows of a wave's (16*MI) x 64 output block, loaded to registers ahead of
// the epilogue (2*MI 16-byte loads, lane layout of epilogue_tp): callers that have the
// VGPRs issue them during the last K-steps so the epilogue never waits on them.
template <typename CT, int MI>
__device__ __forceinline__ void load_residual_tp(const ConvGemmParams& p, u32x4 (&res)[MI][2], int mw, int nw,
                                                 int lane) {
    const int grp = lane >> 4;
    const int c0 = 8 * ((grp & 1) * 2 + (grp >> 1));
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        int m = mw + i * 16 + (lane & 15);
        m = m < p.M ? m : p.M - 1;  // valid address; rows past M are never stored
        const CT* rp = (const CT*)p.R + (int64_t)res_row(p, m) * p.ldr + nw + c0;
        res[i][0] = *(const u32x4*)rp;
        res[i][1] = *(const u32x4*)(rp + 32);
    }
}

// As load_residual_tp, through a buffer resource with 32-bit byte offsets computed at
// the call (the wave's base row is laundered through an empty asm, so the row
// arithmetic is not hoisted out of the K loop and held there in 16 address VGPRs;
// caller: R extent < 2^31 bytes).
template <typename CT, int MI>
__device__ __forceinline__ void load_residual_tp_buf(const ConvGemmParams& p, u32x4 (&res)[MI][2], int mw, int nw,
                                                     int lane) {
    asm volatile("" : "+v"(mw));
    const __amdgpu_buffer_rsrc_t r_rsrc = make_rsrc(p.R, 0x7FFFFFFF);
    const int grp = lane >> 4;
    const int c0 = 8 * ((grp & 1) * 2 + (grp >> 1));
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        int m = mw + i * 16 + (lane & 15);
        m = m < p.M ? m : p.M - 1;  // valid address; rows past M are never stored
        const int off = (res_row(p, m) * p.ldr + nw + c0) * (int)sizeof(CT);
        res[i][0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r_rsrc, off, 0, 0));
        res[i][1] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r_rsrc, off + 64, 0, 0));
    }
}

// PRE: the residual is already in `pre` (load_residual_tp, waited for by the caller).
// HAS_R: -1 = p.R decides at run time; 0 / 1 = known at compile time (straight-line
// code, so the compiler's own vmcnt waits before the residual uses stay counted).
// AUX: cache policy of the output stores (0 = default; 2 = nt, streamed past the caches)
// m_base: the row y_rsrc starts at (callers with outputs past 2^31 bytes rebase the
// resource per tile; store offsets are then tile-relative)
template <typename CT, int MI, bool PRE = false, int HAS_R = -1, int AUX = 0>
__device__ __forceinline__ void epilogue_tp(const ConvGemmParams& p, f32x4 (&acc)[MI][4], int mw, int nw,
                                            int lane, const float* s_scale, const float* s_shift,
                                            __amdgpu_buffer_rsrc_t y_rsrc, const u32x4 (*pre)[2] = nullptr,
                                            int m_base = 0) {
    const int grp = lane >> 4;
    const int c0 = 8 * ((grp & 1) * 2 + (grp >> 1));
    float sc[4][4], sh[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = nw + 16 * j + 4 * grp;
        const f32x4 s4 = *(const f32x4*)&s_scale[n];
        const f32x4 h4 = *(const f32x4*)&s_shift[n];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            sc[j][q] = s4[q];
            sh[j][q] = h4[q];
        }
    }
    const bool has_r = HAS_R < 0 ? p.R != nullptr : HAS_R == 1;
    u32x4 res[2][2];
    auto load_res = [&](int i, u32x4 (&rr)[2]) {
        int m = mw + i * 16 + (lane & 15);
        m = m < p.M ? m : p.M - 1;  // valid address; rows past M are never stored
        const CT* rp = (const CT*)p.R + (int64_t)res_row(p, m) * p.ldr + nw + c0;
        rr[0] = *(const u32x4*)rp;
        rr[1] = *(const u32x4*)(rp + 32);
    };
    if (has_r && !PRE) load_res(0, res[0]);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        const int m = mw + i * 16 + (lane & 15);
        if (has_r && !PRE) {
            // issue order per block: res(i+1), [wait res(i)], stores(i)
            if (i + 1 < MI) load_res(i + 1, res[(i + 1) & 1]);
            if (i == 0)
                vm_wait_n<2>();
            else if (i + 1 < MI)
                vm_wait_n<4>();
            else
                vm_wait_n<2>();
        }
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
            float v[8];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                float x = __fadd_rn(__fmul_rn(acc[i][2 * jp][d], sc[2 * jp][d]), sh[2 * jp][d]);
                float y = __fadd_rn(__fmul_rn(acc[i][2 * jp + 1][d], sc[2 * jp + 1][d]), sh[2 * jp + 1][d]);
                if (p.relu) {
                    x = x > 0.f ? x : 0.f;
                    y = y > 0.f ? y : 0.f;
                }
                // odd 16-lane rows of x <-> even rows of y.  Inline asm: hipcc 7.2 folds
                // repeated __builtin_amdgcn_permlane16_swap calls on different operands
                // into one (miscompile); x, y were just written by VALU -> 2 wait states
                asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
                v[d] = x;
                v[d + 4] = y;
            }
            typedef CT ct8 __attribute__((ext_vector_type(8)));
            if (has_r) {
                const ct8 r8 = __builtin_bit_cast(ct8, PRE ? pre[i][jp] : res[i & 1][jp]);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] += (float)r8[e];
            }
            ct8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = (CT)v[e];
            const uint32_t yo = m < p.M ? (uint32_t)(((size_t)(m - m_base) * p.ldy + nw + 32 * jp + c0) * sizeof(CT))
                                        : 0xFFFFFFF0u;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), y_rsrc, yo, 0, AUX);
        }
    }
}

// epilogue_tp with the residual of row block i fetched by `res_of(i, rr)` from rows already on
// chip (conv_gemm_a4: landed in LDS by LDS-DMA during the last K-tiles), so no vmcnt waits
// here; the same arithmetic, so the same bits as epilogue_tp.
template <typename CT, int MI, typename RF>
__device__ __forceinline__ void epilogue_tp_rf(const ConvGemmParams& p, f32x4 (&acc)[MI][4], int mw, int nw,
                                               int lane, const float* s_scale, const float* s_shift,
                                               __amdgpu_buffer_rsrc_t y_rsrc, int m_base, RF&& res_of) {
    const int grp = lane >> 4;
    const int c0 = 8 * ((grp & 1) * 2 + (grp >> 1));
    float sc[4][4], sh[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = nw + 16 * j + 4 * grp;
        const f32x4 s4 = *(const f32x4*)&s_scale[n];
        const f32x4 h4 = *(const f32x4*)&s_shift[n];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            sc[j][q] = s4[q];
            sh[j][q] = h4[q];
        }
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        const int m = mw + i * 16 + (lane & 15);
        u32x4 rr[2];
        res_of(i, rr);
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
            float v[8];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                float x = __fadd_rn(__fmul_rn(acc[i][2 * jp][d], sc[2 * jp][d]), sh[2 * jp][d]);
                float y = __fadd_rn(__fmul_rn(acc[i][2 * jp + 1][d], sc[2 * jp + 1][d]), sh[2 * jp + 1][d]);
                if (p.relu) {
                    x = x > 0.f ? x : 0.f;
                    y = y > 0.f ? y : 0.f;
                }
                asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
                v[d] = x;
                v[d + 4] = y;
            }
            typedef CT ct8 __attribute__((ext_vector_type(8)));
            const ct8 r8 = __builtin_bit_cast(ct8, rr[jp]);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += (float)r8[e];
            ct8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = (CT)v[e];
            const uint32_t yo = m < p.M ? (uint32_t)(((size_t)(m - m_base) * p.ldy + nw + 32 * jp + c0) * sizeof(CT))
                                        : 0xFFFFFFF0u;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), y_rsrc, yo, 0, 0);
        }
    }
}

// epilogue_tp for the split-fp16 path (VP3D_DTYPE_F16X3, conv_gemm_q64<_, _, X3>): rows of
// split activations hold channel n's halves at 64 (n / 32) + n % 32 (hi) and +32 (lo), so
// a lane's 8 channels nw + 32 jp + c0 + 0..7 are 16 bytes of hi and, 64 bytes on, 16 of lo.
// Residual (block input, split): hi + lo rebuilt in f32 and added as one value (the
// reference's res + relu(bn(conv)), TemporalModel.py:135,195).  Output: split (hi =
// f16(v), lo = f16(v - hi)) or, OUT_F32, the f32 row for the exact f32 shrink GEMM.
// 4 residual loads and 4 stores per row block: the waits count both.
// Split-fp16 epilogue arithmetic on channel pairs as mixed-precision FMAs (the f16 sources widen
// exactly, one rounding per result -- the same bits as the convert / f32 add / convert forms, in
// fewer instructions):
//   x3_res_sum2: a residual pair's hi + lo (f16 pairs, one dword each) as two exact f32 sums
//   x3_split_lo2: the lo halves of an f32 pair whose hi halves (packed f16) are h: f16(x - hi),
//                 written as one packed pair (v_fma_mixlo_f16 / v_fma_mixhi_f16)
__device__ __forceinline__ void x3_res_sum2(uint32_t rh, uint32_t rl, float& t0, float& t1) {
    asm("v_fma_mix_f32 %0, %2, 1.0, %3 op_sel_hi:[1,0,1]\n\t"
        "v_fma_mix_f32 %1, %2, 1.0, %3 op_sel:[1,0,1] op_sel_hi:[1,0,1]"
        : "=&v"(t0), "=v"(t1)
        : "v"(rh), "v"(rl));
}
__device__ __forceinline__ uint32_t x3_split_lo2(uint32_t h, float x0, float x1) {
    uint32_t r;
    asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
        "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
        : "=&v"(r)
        : "v"(h), "v"(x0), "v"(x1));
    return r;
}
// f32 pair -> packed f16 pair (round to nearest even, one v_cvt_pk_f16_f32)
__device__ __forceinline__ uint32_t x3_hi2(float x0, float x1) {
    typedef float f2_ __attribute__((ext_vector_type(2)));
    typedef _Float16 h2_ __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2_{x0, x1}, h2_));
}

// f16x3 range guard.  A value split into f16 halves must satisfy |x| <= 65,504: past it hi =
// inf and every later product is inf / NaN (or, through the integer-max ReLU, silently 0).
// The split epilogues fold |x| of what they split into a running max (x3_absmax2: one
// v_max3_f32 per pair); at the end of a tile a lane over the range ORs kFaultNonFinite into
// the handle's fault word, whose device address the host keeps just past the layer's
// scale_x3 vector (Layer::scale_x3[N .. N + 1], vp3d_capi.cpp upload_weights).
__device__ __forceinline__ float x3_absmax2(float m, float a, float b) {
    // (as asm: the compiler's fmaxf form canonicalises each operand first, 3 instructions)
    float r;
    asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}
// the input rows' check, on the packed hi halves: |hi| >= 0x7C00 is inf or NaN (what the
// split of a value past the range, or of a NaN, leaves); one v_pk_max_u16 per pair
__device__ __forceinline__ uint32_t x3_himax2(uint32_t m, uint32_t h) {
    typedef unsigned short u16x2_ __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2_, m),
                                                                  __builtin_bit_cast(u16x2_, h & 0x7FFF7FFFu)));
}
__device__ __forceinline__ bool x3_hi_bad(uint32_t m) { return (m & 0xFFFFu) >= 0x7C00u || (m >> 16) >= 0x7C00u; }
__device__ __forceinline__ void x3_range_flag(float m, const float* scale_x3, int n) {
    if (__builtin_expect(!(m <= 65504.f), 0)) {  // (a NaN input compares false too)
        unsigned* const f = *(unsigned* const*)(scale_x3 + n);
        if (f) __hip_atomic_fetch_or(f, kFaultNonFinite, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <bool OUT_F32, int HAS_R>
__device__ __forceinline__ void epilogue_tp_x3(const ConvGemmParams& p, f32x4 (&acc)[8][4], int mw, int nw, int lane,
                                               const float* s_scale, const float* s_shift,
                                               __amdgpu_buffer_rsrc_t y_rsrc, int m_base) {
    constexpr int MI = 8;
    const int grp = lane >> 4;
    const int c0 = 8 * ((grp & 1) * 2 + (grp >> 1));
    float sc[4][4], sh[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = nw + 16 * j + 4 * grp;
        const f32x4 s4 = *(const f32x4*)&s_scale[n];
        const f32x4 h4 = *(const f32x4*)&s_shift[n];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            sc[j][q] = s4[q];
            sh[j][q] = h4[q];
        }
    }
    u32x4 res[2][2][2];  // [row block parity][jp][hi, lo]
    auto load_res = [&](int i, u32x4 (&rr)[2][2]) {
        int m = mw + i * 16 + (lane & 15);
        m = m < p.M ? m : p.M - 1;  // valid address; rows past M are never stored
        const f16* rp = (const f16*)p.R + (int64_t)res_row(p, m) * p.ldr + 2 * nw + c0;
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
            rr[jp][0] = *(const u32x4*)(rp + 64 * jp);
            rr[jp][1] = *(const u32x4*)(rp + 64 * jp + 32);
        }
    };
    if (HAS_R) load_res(0, res[0]);
    float vmax = 0.f;  // |x| over what this tile splits (x3_range_flag)
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        const int m = mw + i * 16 + (lane & 15);
        if (HAS_R) {
            // issue order per block: res(i+1) (4 loads), [wait res(i)], stores(i) (4)
            if (i + 1 < MI) load_res(i + 1, res[(i + 1) & 1]);
            if (i == 0)
                vm_wait_n<4>();
            else if (i + 1 < MI)
                vm_wait_n<8>();
            else
                vm_wait_n<4>();
        }
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
            float v[8];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                float x = __fadd_rn(__fmul_rn(acc[i][2 * jp][d], sc[2 * jp][d]), sh[2 * jp][d]);
                float y = __fadd_rn(__fmul_rn(acc[i][2 * jp + 1][d], sc[2 * jp + 1][d]), sh[2 * jp + 1][d]);
                if (p.relu) {
                    x = x > 0.f ? x : 0.f;
                    y = y > 0.f ? y : 0.f;
                }
                asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
                v[d] = x;
                v[d + 4] = y;
            }
            if (HAS_R) {
                // v + (rh + rl): the exact pair sums as mixed FMAs, then one f32 add each
                const u32x4 rh = res[i & 1][jp][0], rl = res[i & 1][jp][1];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float t0, t1;
                    gemm::x3_res_sum2(rh[e], rl[e], t0, t1);
                    v[2 * e] += t0;
                    v[2 * e + 1] += t1;
                }
            }
            const bool in = m < p.M;
            if constexpr (OUT_F32) {
                const uint32_t yo = in ? (uint32_t)(((size_t)(m - m_base) * p.ldy + nw + 32 * jp + c0) * 4) : 0xFFFFFFE0u;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f32x4{v[0], v[1], v[2], v[3]}),
                                                       y_rsrc, yo, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f32x4{v[4], v[5], v[6], v[7]}),
                                                       y_rsrc, yo + 16, 0, 0);
            } else {
                // hi = f16(v), lo = f16(v - hi) (v_fma_mixlo/mixhi: one rounding, as before)
                u32x4 oh, ol;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    oh[e] = gemm::x3_hi2(v[2 * e], v[2 * e + 1]);
                    ol[e] = gemm::x3_split_lo2(oh[e], v[2 * e], v[2 * e + 1]);
                    if (in) vmax = x3_absmax2(vmax, v[2 * e], v[2 * e + 1]);
                }
                const uint32_t yo = in ? (uint32_t)(((size_t)(m - m_base) * p.ldy + 2 * nw + 64 * jp + c0) * 2)
                                       : 0xFFFFFF00u;
                __builtin_amdgcn_raw_buffer_store_b128(oh, y_rsrc, yo, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(ol, y_rsrc, yo + 64, 0, 0);
            }
        }
    }
    if constexpr (!OUT_F32) x3_range_flag(vmax, p.scale, p.N);
}

}  // namespace gemm
}  // namespace vp3d
