// Temporal-convolution GEMM kernels for gfx950 (MI355X, CDNA4).
//
// Every convolution of TemporalModel / TemporalModelOptimized1f
// (reference common/models/TemporalModel.py:102,113-119,168,179-181,33) runs
// through one implicit-GEMM kernel family over channel-last activations; see
// ConvGemmParams in kernels.h for the row mapping.  The BatchNorm (eval, folded
// to a per-channel scale/shift), ReLU, dropout (identity in eval) and the
// residual slice-add of TemporalModel.py:127-135 / :189-195 are the epilogue.
//
// Geometry (both families): 256 threads = 4 waves in a 2x2 arrangement, a
// 128x128 output tile per workgroup, each wave 64x64 = 4x4 MFMA 16x16 blocks.
// Operands are staged global -> registers -> LDS (double buffered, one barrier
// per K-step), with an XOR swizzle on 16-byte chunks that makes every
// ds_read_b128 fragment read bank-conflict free (checked against the gfx950
// ds_read_b128 lane groups).  Workgroups are remapped so that the 8 N-tiles of
// an M-panel run on one XCD (shared A panel in that XCD's L2).
//
//  * 16-bit family: v_mfma_f32_16x16x32_{bf16,f16}, BK = 64, 128-byte LDS rows,
//    chunk' = chunk ^ (row & 7).
//  * f32 family:    v_mfma_f32_16x16x4_f32 (exact f32 fmaf chain), BK = 16,
//    64-byte LDS rows, chunk' = (chunk + 2*((row>>2)&3)) & 3.  Lane l reads the
//    4 consecutive k of its row in one ds_read_b128 and feeds them to 4
//    successive MFMAs (k = 4*(l>>4) + s); A and B use the same k permutation,
//    so the dot product is unchanged.
#include "kernels.h"

namespace vp3d {
namespace {

typedef __bf16 bf16;
typedef _Float16 f16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128;
constexpr int BN = 128;

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

// Scalar A element loader (general tap mapping, bounds-checked, zero fill).
template <typename AT>
__device__ __forceinline__ float load_a_scalar(const ConvGemmParams& p, int srow, int kk) {
    if (kk >= p.K) return 0.f;
    const int tap = kk / p.Ktap;
    const int c = kk - tap * p.Ktap;
    const AT* A = (const AT*)p.A;
    return to_f32(A[(int64_t)(srow + tap * p.dil) * p.lda + c]);
}

// Epilogue for one accumulator register: BN scale/shift, ReLU, residual add, store.
template <typename OT>
__device__ __forceinline__ void epi_store(const ConvGemmParams& p, int m, int n, float v,
                                          float sc, float sh) {
    // BatchNorm eval as ATen's CPU kernel evaluates it: x * alpha + beta, two roundings
    v = __fadd_rn(__fmul_rn(v, sc), sh);
    if (p.relu) v = v > 0.f ? v : 0.f;
    if (p.R) v += to_f32(((const OT*)p.R)[(int64_t)res_row(p, m) * p.ldr + n]);
    ((OT*)p.Y)[(int64_t)m * p.ldy + n] = from_f32<OT>(v);
}

// ---------------------------------------------------------------------------
// 16-bit operand family
// ---------------------------------------------------------------------------
template <typename AT, typename OT, typename CT, bool AVEC>
__global__ __launch_bounds__(256) void conv_gemm_h16(ConvGemmParams p) {
    constexpr int BK = 64;                    // 8 chunks of 8 elements per row
    __shared__ __attribute__((aligned(16))) u32x4 smem[2][2][BM * BK / 8];  // [buf][A,B]

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wr = wid >> 1, wc = wid & 1;

    const int ntn = (p.N + BN - 1) / BN;
    const int ntm = (p.M + BM - 1) / BM;
    const int wg = xcd_remap(blockIdx.x, ntm * ntn);
    const int tile_m = wg / ntn;
    const int tile_n = wg - tile_m * ntn;
    const int m0 = tile_m * BM, n0 = tile_n * BN;

    // staging assignment: 1024 chunks of 16 bytes per operand tile, 4 per thread
    const int ld_row = tid >> 3;  // + 32*i
    const int ld_c = tid & 7;
    int srow[4];
    bool mval[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + ld_row + 32 * i;
        mval[i] = m < p.M;
        srow[i] = mval[i] ? src_row(p, m) : 0;
    }
    const CT* Wp = (const CT*)p.W;

    u32x4 ra[4], rb[4];
    auto gload = [&](int k0) {
        // A
        if constexpr (AVEC) {
            const int tap = k0 / p.Ktap;
            const int cin = k0 - tap * p.Ktap + ld_c * 8;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (mval[i]) {
                    const int64_t off = (int64_t)(srow[i] + tap * p.dil) * p.lda + cin;
                    if constexpr (sizeof(AT) == 2) {
                        ra[i] = *(const u32x4*)((const AT*)p.A + off);
                    } else {
                        const f32x4 x0 = *(const f32x4*)((const float*)p.A + off);
                        const f32x4 x1 = *(const f32x4*)((const float*)p.A + off + 4);
                        float v[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
                        ra[i] = pack8<CT>(v);
                    }
                } else {
                    ra[i] = u32x4{0u, 0u, 0u, 0u};
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e)
                    v[e] = mval[i] ? load_a_scalar<AT>(p, srow[i], k0 + ld_c * 8 + e) : 0.f;
                ra[i] = pack8<CT>(v);
            }
        }
        // B (padded to [Np][Kp], always in bounds)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int n = n0 + ld_row + 32 * i;
            rb[i] = *(const u32x4*)(Wp + (int64_t)n * p.Kp + k0 + ld_c * 8);
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = ld_row + 32 * i;
            const int slot = r * 8 + (ld_c ^ (r & 7));
            smem[buf][0][slot] = ra[i];
            smem[buf][1][slot] = rb[i];
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = p.Kp / BK;
    gload(0);
    lstore(0);
    __syncthreads();

    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
        const bool more = kt + 1 < nk;
        if (more) gload((kt + 1) * BK);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            u32x4 af[4], bfm[4];
            const int c = ks * 4 + (lane >> 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = wr * 64 + i * 16 + (lane & 15);
                af[i] = smem[cur][0][r * 8 + (c ^ (r & 7))];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = wc * 64 + j * 16 + (lane & 15);
                bfm[j] = smem[cur][1][r * 8 + (c ^ (r & 7))];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = mfma16<CT>(af[i], bfm[j], acc[i][j]);
        }
        if (more) lstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }

    // epilogue: D(row = (lane>>4)*4 + r, col = lane & 15) of each 16x16 block
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = n0 + wc * 64 + j * 16 + (lane & 15);
        if (n >= p.N) continue;
        const float sc = p.scale[n], sh = p.shift[n];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wr * 64 + i * 16 + (lane >> 4) * 4 + r;
                if (m < p.M) epi_store<OT>(p, m, n, acc[i][j][r], sc, sh);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// exact f32 family
// ---------------------------------------------------------------------------
template <bool AVEC>
__global__ __launch_bounds__(256) void conv_gemm_f32(ConvGemmParams p) {
    constexpr int BK = 16;  // 4 chunks of 4 floats per row
    __shared__ __attribute__((aligned(16))) f32x4 smem[2][2][BM * BK / 4];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wr = wid >> 1, wc = wid & 1;

    const int ntn = (p.N + BN - 1) / BN;
    const int ntm = (p.M + BM - 1) / BM;
    const int wg = xcd_remap(blockIdx.x, ntm * ntn);
    const int tile_m = wg / ntn;
    const int tile_n = wg - tile_m * ntn;
    const int m0 = tile_m * BM, n0 = tile_n * BN;

    // 512 chunks per operand tile, 2 per thread
    const int ld_row = tid >> 2;  // + 64*i
    const int ld_c = tid & 3;
    int srow[2];
    bool mval[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int m = m0 + ld_row + 64 * i;
        mval[i] = m < p.M;
        srow[i] = mval[i] ? src_row(p, m) : 0;
    }
    const float* Wp = (const float*)p.W;
    const float* A = (const float*)p.A;

    f32x4 ra[2], rb[2];
    auto gload = [&](int k0) {
        if constexpr (AVEC) {
            const int tap = k0 / p.Ktap;
            const int cin = k0 - tap * p.Ktap + ld_c * 4;
#pragma unroll
            for (int i = 0; i < 2; ++i)
                ra[i] = mval[i] ? *(const f32x4*)(A + (int64_t)(srow[i] + tap * p.dil) * p.lda + cin)
                                : f32x4{0.f, 0.f, 0.f, 0.f};
        } else {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    ra[i][e] = mval[i] ? load_a_scalar<float>(p, srow[i], k0 + ld_c * 4 + e) : 0.f;
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int n = n0 + ld_row + 64 * i;
            rb[i] = *(const f32x4*)(Wp + (int64_t)n * p.Kp + k0 + ld_c * 4);
        }
    };
    auto swz = [](int r, int c) { return r * 4 + ((c + 2 * ((r >> 2) & 3)) & 3); };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int r = ld_row + 64 * i;
            smem[buf][0][swz(r, ld_c)] = ra[i];
            smem[buf][1][swz(r, ld_c)] = rb[i];
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = p.Kp / BK;
    gload(0);
    lstore(0);
    __syncthreads();
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
        const bool more = kt + 1 < nk;
        if (more) gload((kt + 1) * BK);
        f32x4 af[4], bfm[4];
        const int c = lane >> 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = smem[cur][0][swz(wr * 64 + i * 16 + (lane & 15), c)];
#pragma unroll
        for (int j = 0; j < 4; ++j) bfm[j] = smem[cur][1][swz(wc * 64 + j * 16 + (lane & 15), c)];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s], bfm[j][s], acc[i][j], 0, 0, 0);
        if (more) lstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }

#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = n0 + wc * 64 + j * 16 + (lane & 15);
        if (n >= p.N) continue;
        const float sc = p.scale[n], sh = p.shift[n];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wr * 64 + i * 16 + (lane >> 4) * 4 + r;
                if (m < p.M) epi_store<float>(p, m, n, acc[i][j][r], sc, sh);
            }
    }
}

template <typename AT, typename OT, typename CT>
hipError_t launch_h16(const ConvGemmParams& p, bool avec, dim3 grid, hipStream_t s) {
    if (avec)
        hipLaunchKernelGGL((conv_gemm_h16<AT, OT, CT, true>), grid, dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL((conv_gemm_h16<AT, OT, CT, false>), grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

template <typename CT>
hipError_t launch_h16_dispatch(const ConvGemmParams& p, Act a, Act o, bool avec, dim3 grid,
                               hipStream_t s) {
    if (a == Act::F32 && o == Act::F32) return launch_h16<float, float, CT>(p, avec, grid, s);
    if (a == Act::F32) return launch_h16<float, CT, CT>(p, avec, grid, s);
    if (o == Act::F32) return launch_h16<CT, float, CT>(p, avec, grid, s);
    return launch_h16<CT, CT, CT>(p, avec, grid, s);
}

}  // namespace

hipError_t launch_conv_gemm(const ConvGemmParams& p, Act a_type, Act out_type, Act compute,
                            hipStream_t stream) {
    if (p.M <= 0 || p.N <= 0) return hipSuccess;
    const int ntm = (p.M + BM - 1) / BM;
    const int ntn = (p.N + BN - 1) / BN;
    const dim3 grid(ntm * ntn);
    if (compute == Act::F32) {
        if (a_type != Act::F32 || out_type != Act::F32) return hipErrorInvalidValue;
        const bool avec = (p.Ktap % 16 == 0) && (p.lda % 4 == 0) &&
                          ((reinterpret_cast<uintptr_t>(p.A) & 15) == 0);
        if (avec)
            hipLaunchKernelGGL((conv_gemm_f32<true>), grid, dim3(256), 0, stream, p);
        else
            hipLaunchKernelGGL((conv_gemm_f32<false>), grid, dim3(256), 0, stream, p);
        return hipGetLastError();
    }
    if (a_type != Act::F32 && a_type != compute) return hipErrorInvalidValue;
    if (out_type != Act::F32 && out_type != compute) return hipErrorInvalidValue;
    const bool avec = (p.Ktap % 64 == 0) && (p.lda % 8 == 0) &&
                      ((reinterpret_cast<uintptr_t>(p.A) & 15) == 0);
    if (compute == Act::BF16) return launch_h16_dispatch<bf16>(p, a_type, out_type, avec, grid, stream);
    return launch_h16_dispatch<f16>(p, a_type, out_type, avec, grid, stream);
}

}  // namespace vp3d
