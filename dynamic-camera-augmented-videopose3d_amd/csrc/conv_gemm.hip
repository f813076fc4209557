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
#include <cstdlib>
#include <cstring>

#include "gemm_common.h"

namespace vp3d {
namespace {

using namespace gemm;

constexpr int BM = 128;
constexpr int BN = 128;

// ---------------------------------------------------------------------------
// 16-bit operand family
// ---------------------------------------------------------------------------
constexpr int kH16Bk = 64;
constexpr int kH16MainBytes = 2 * 2 * BM * kH16Bk * 2;        // [buf][A,B] bf16 tiles
constexpr int kEpiBytes = 4 * 64 * kEpiLd * 4;                // 4 waves x 64 rows
constexpr int kH16Smem = kH16MainBytes > kEpiBytes ? kH16MainBytes : kEpiBytes;

template <typename AT, typename OT, typename CT, int AMODE, bool VEPI>
__global__ __launch_bounds__(256) void conv_gemm_h16(ConvGemmParams p) {
    constexpr int BK = kH16Bk;  // 8 chunks of 8 elements per row
    __shared__ __attribute__((aligned(16))) char smem_raw[kH16Smem];
    u32x4* const s4 = (u32x4*)smem_raw;  // [buf][A,B][BM*BK/8]
    constexpr int TILE = BM * BK / 8;

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
        if constexpr (AMODE == A_VEC) {
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
                load_a_run<AT, AMODE, 8>(p, srow[i], k0 + ld_c * 8, mval[i], v);
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
            s4[(2 * buf) * TILE + slot] = ra[i];
            s4[(2 * buf + 1) * TILE + slot] = rb[i];
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
                af[i] = s4[(2 * cur) * TILE + r * 8 + (c ^ (r & 7))];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = wc * 64 + j * 16 + (lane & 15);
                bfm[j] = s4[(2 * cur + 1) * TILE + r * 8 + (c ^ (r & 7))];
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

    const int mw = m0 + wr * 64, nw = n0 + wc * 64;
    if constexpr (VEPI)
        epilogue_vec<OT, 4, 64>(p, acc, (float*)smem_raw + wid * 64 * kEpiLd, mw, nw, lane);
    else
        epilogue_scalar<OT, 4>(p, acc, mw, nw, lane);
}

// ---------------------------------------------------------------------------
// exact f32 family
// ---------------------------------------------------------------------------
constexpr int kF32Bk = 16;
constexpr int kF32MainBytes = 2 * 2 * BM * kF32Bk * 4;
constexpr int kF32EpiBytes = 4 * 32 * kEpiLd * 4;  // two passes of 32 rows per wave
constexpr int kF32Smem = kF32MainBytes > kF32EpiBytes ? kF32MainBytes : kF32EpiBytes;

template <int AMODE, bool VEPI>
__global__ __launch_bounds__(256) void conv_gemm_f32(ConvGemmParams p) {
    constexpr int BK = kF32Bk;  // 4 chunks of 4 floats per row
    __shared__ __attribute__((aligned(16))) char smem_raw[kF32Smem];
    f32x4* const s4 = (f32x4*)smem_raw;  // [buf][A,B][BM*BK/4]
    constexpr int TILE = BM * BK / 4;

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
        if constexpr (AMODE == A_VEC) {
            const int tap = k0 / p.Ktap;
            const int cin = k0 - tap * p.Ktap + ld_c * 4;
#pragma unroll
            for (int i = 0; i < 2; ++i)
                ra[i] = mval[i] ? *(const f32x4*)(A + (int64_t)(srow[i] + tap * p.dil) * p.lda + cin)
                                : f32x4{0.f, 0.f, 0.f, 0.f};
        } else {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                float v[4];
                load_a_run<float, AMODE, 4>(p, srow[i], k0 + ld_c * 4, mval[i], v);
                ra[i] = f32x4{v[0], v[1], v[2], v[3]};
            }
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
            s4[(2 * buf) * TILE + swz(r, ld_c)] = ra[i];
            s4[(2 * buf + 1) * TILE + swz(r, ld_c)] = rb[i];
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
        for (int i = 0; i < 4; ++i) af[i] = s4[(2 * cur) * TILE + swz(wr * 64 + i * 16 + (lane & 15), c)];
#pragma unroll
        for (int j = 0; j < 4; ++j) bfm[j] = s4[(2 * cur + 1) * TILE + swz(wc * 64 + j * 16 + (lane & 15), c)];
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

    const int mw = m0 + wr * 64, nw = n0 + wc * 64;
    if constexpr (VEPI)
        epilogue_vec<float, 4, 32>(p, acc, (float*)smem_raw + wid * 32 * kEpiLd, mw, nw, lane);
    else
        epilogue_scalar<float, 4>(p, acc, mw, nw, lane);
}

template <typename AT, typename OT, typename CT, int AMODE>
hipError_t launch_h16_v(const ConvGemmParams& p, bool vepi, dim3 grid, hipStream_t s) {
    if (vepi)
        hipLaunchKernelGGL((conv_gemm_h16<AT, OT, CT, AMODE, true>), grid, dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL((conv_gemm_h16<AT, OT, CT, AMODE, false>), grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

template <typename AT, typename OT, typename CT>
hipError_t launch_h16(const ConvGemmParams& p, int amode, bool vepi, dim3 grid, hipStream_t s) {
    if (amode == A_VEC) return launch_h16_v<AT, OT, CT, A_VEC>(p, vepi, grid, s);
    if constexpr (sizeof(AT) == 4)
        if (amode == A_PAIRS) return launch_h16_v<AT, OT, CT, A_PAIRS>(p, vepi, grid, s);
    return launch_h16_v<AT, OT, CT, A_SCALAR>(p, vepi, grid, s);
}

template <typename CT>
hipError_t launch_h16_dispatch(const ConvGemmParams& p, Act a, Act o, int amode, bool vepi,
                               dim3 grid, hipStream_t s) {
    if (a == Act::F32 && o == Act::F32) return launch_h16<float, float, CT>(p, amode, vepi, grid, s);
    if (a == Act::F32) return launch_h16<float, CT, CT>(p, amode, vepi, grid, s);
    if (o == Act::F32) return launch_h16<CT, float, CT>(p, amode, vepi, grid, s);
    return launch_h16<CT, CT, CT>(p, amode, vepi, grid, s);
}

template <int AMODE>
hipError_t launch_f32(const ConvGemmParams& p, bool vepi, dim3 grid, hipStream_t s) {
    if (vepi)
        hipLaunchKernelGGL((conv_gemm_f32<AMODE, true>), grid, dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL((conv_gemm_f32<AMODE, false>), grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

// Which 256x256 kernel a large layer runs on:
//   default: every tap-aligned layer with >= 384 tiles on the one-wave-per-SIMD AGPR kernel
//   (conv_gemm_a4.hip; block 1 at B = 65,536, same box: k3 8.61-8.64 vs 9.14-9.19 ms on q64,
//   1x1 + residual 3.57-3.68 vs 4.23; the dilated k3 convs of sequence mode 0.34 vs 0.39 ms on
//   the LDS-ring kernel; bit-identical to q64), then the 64-deep quadrant-phase kernel
//   (conv_gemm_q64.hip) and the ping-pong kernel (conv_gemm_8p.hip) where a4 is not eligible,
//   the LDS-ring kernel (conv_gemm_big.hip) for the dilated layers a4 does not take.
//   VP3D_GEMM=a4 / q64 / 8p -> that kernel wherever eligible (q64 / 8p: dilated layers included),
//   VP3D_GEMM=big -> the LDS-ring kernel everywhere; the override tests run each.
//   VP3D_GEMM=h16 -> the 128x128 kernel everywhere (measurement).
//   The round-1 A/B schedules (persistent, dynamic-queue, older ping-pong, transposed
//   persistent) were 3-10 % slower and live outside the library, in tools/ubench/retired/.
//   Read at every launch (a getenv per layer is noise next to the kernel), so a test can
//   flip it within one process.
int gemm_8p_mode() {
    const char* e = getenv("VP3D_GEMM");
    if (!e) return 1;
    if (strcmp(e, "8p") == 0) return 2;
    if (strcmp(e, "q64") == 0) return 3;
    if (strcmp(e, "h16") == 0) return 4;  // the 128x128 kernel everywhere (measurement)
    if (strcmp(e, "a4") == 0) return 5;   // the one-wave-per-SIMD AGPR kernel where eligible
    return strcmp(e, "big") == 0 ? 0 : 1;
}
bool gemm_8p_env(const ConvGemmParams& p) {
    const int m = gemm_8p_mode();
    return m == 2 || (m == 1 && p.dil == 1);
}

bool aligned(const void* ptr, uintptr_t a) { return (reinterpret_cast<uintptr_t>(ptr) & (a - 1)) == 0; }


// ---------------------------------------------------------------------------
// narrow layers (N <= 64: the shrink conv, TemporalModel.py:33 / :74) on the 16-bit
// path: one workgroup per 16 rows x 64 output channels, K streamed straight from global
// memory into MFMA fragments (the 16-bit weights, <= 128 KiB, stay in L2), f32 out.
// The 128x128 tile would give the whole layer only M/128 workgroups.
// ---------------------------------------------------------------------------
template <typename CT>
__global__ __launch_bounds__(256) void conv_gemm_narrow(ConvGemmParams p) {
    // 4 waves split K four ways (short dependent load->MFMA chains), partial 16x64
    // tiles summed through LDS by wave 0
    __shared__ float red[3][16][65];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int m0 = blockIdx.x * 16;
    const int r = lane & 15, kc = (lane >> 4) * 8;
    const int m = m0 + r;
    const bool mv = m < p.M;
    const CT* arow = (const CT*)p.A + (int64_t)(mv ? src_row(p, m) : 0) * p.lda;
    const CT* W = (const CT*)p.W;
    const int ksteps = p.K / 32;
    const int kb = (ksteps * wid) / 4, ke = (ksteps * (wid + 1)) / 4;
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ks = kb; ks < ke; ks += 2) {
        const bool two = ks + 1 < ke;
        const int k0 = ks * 32;
        u32x4 a0 = mv ? *(const u32x4*)(arow + k0 + kc) : u32x4{0, 0, 0, 0};
        u32x4 a1 = (mv && two) ? *(const u32x4*)(arow + k0 + 32 + kc) : u32x4{0, 0, 0, 0};
        u32x4 b0[4], b1[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            b0[j] = *(const u32x4*)(W + (int64_t)(j * 16 + r) * p.Kp + k0 + kc);
            b1[j] = two ? *(const u32x4*)(W + (int64_t)(j * 16 + r) * p.Kp + k0 + 32 + kc) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = mfma16<CT>(a0, b0[j], acc[j]);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = mfma16<CT>(a1, b1[j], acc[j]);
    }
    // D[i = 4*(lane/16) + q][n = j*16 + lane%16]
    if (wid > 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) red[wid - 1][(lane >> 4) * 4 + q][j * 16 + r] = acc[j][q];
    }
    __syncthreads();
    if (wid != 0) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = j * 16 + r;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = (lane >> 4) * 4 + q;
            float v = acc[j][q];
            v = v + red[0][i][n];
            v = v + red[1][i][n];
            v = v + red[2][i][n];
            const int mm = m0 + i;
            if (n < p.N && mm < p.M) epi_store<float>(p, mm, n, v, p.scale[n], p.shift[n]);
        }
    }
}

// Exact-f32 narrow layers (N <= 64: the shrink conv of the fp32 and split-fp16 paths,
// TemporalModel.py:33 / :74; the sequence lifters' 51-wide output Linear): one workgroup per 16
// rows, one wave per 16 of its <= 64 columns, operands straight from global memory (each lane: a
// 16-byte run of its row's K and of its weight row -- the weight rows stay in L1/L2), the MFMA k order of
// conv_gemm_f32 (v_mfma_f32_16x16x4_f32 s = 0..3 over the 16-deep step, lane group c holding
// k = 16 kt + 4 c + s), so the same bits.  conv_gemm_f32 ran these on 128 x 128 tiles: 64 of
// them at B = 8,192 windows, a 64-step K loop with a barrier per step on 64 CUs: 93 vs 54 us,
// and 38 us with an 8-step operand ring (profiles/r04final_narrow_shrink_ring_ab.txt).  From 256
// tiles of 128 rows on, the tile kernel keeps up (B = 65,536: 0.167 vs 0.163 ms narrow).
__global__ __launch_bounds__(256) void conv_gemm_f32_narrow(ConvGemmParams p) {
    // (round 5) one wave per 16 rows x 16 columns: the 4 waves of a workgroup take the 4
    // column blocks of the same 16 rows (A from L1 for three of them), 4x the waves in flight
    // for the loads' latency; each output's MFMA chain unchanged, so the same bits
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (16 * wid >= p.N) return;  // (wave-uniform) no columns in this block
    const int c = lane >> 4, r = lane & 15;
    const int m0 = blockIdx.x * 16;
    const int m = m0 + r;
    const bool mv = m < p.M;
    const float* const arow = (const float*)p.A + (int64_t)(mv ? src_row(p, m) : 0) * p.lda + 4 * c;
    const int n = 16 * wid + r;
    const bool nv = n < p.N;
    const float* const wrow = (const float*)p.W + (int64_t)(nv ? n : 0) * p.Kp + 4 * c;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = p.K / 16;
    // a ring of kDepth K-steps of operands in flight: one step's 4 MFMAs are far shorter than a
    // global load (B = 8,192 with one wave per 64 columns and one step of prefetch: 54 us)
    constexpr int kDepth = 16;
    f32x4 ab[kDepth], wb[kDepth];
    auto load_step = [&](int kt, f32x4& a, f32x4& w) __attribute__((always_inline)) {
        a = mv ? *(const f32x4*)(arow + 16 * kt) : f32x4{0.f, 0.f, 0.f, 0.f};
        w = nv ? *(const f32x4*)(wrow + 16 * kt) : f32x4{0.f, 0.f, 0.f, 0.f};
    };
#pragma unroll
    for (int d = 0; d < kDepth; ++d)
        if (d < nk) load_step(d, ab[d], wb[d]);
    for (int kt0 = 0; kt0 < nk; kt0 += kDepth) {
#pragma unroll
        for (int d = 0; d < kDepth; ++d) {
            const int kt = kt0 + d;
            if (kt < nk) {
#pragma unroll
                for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ab[d][s], wb[d][s], acc, 0, 0, 0);
                if (kt + kDepth < nk) load_step(kt + kDepth, ab[d], wb[d]);
            }
        }
    }
    // epilogue_scalar's mapping for this column block: column n, rows m0 + 4 c + q
    if (nv) {
        const float sc = p.scale[n], sh = p.shift[n];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int mm = m0 + 4 * c + q;
            if (mm < p.M) epi_store<float>(p, mm, n, acc[q], sc, sh);
        }
    }
}

// VP3D_F32_NARROW=0 (measurement; read at every launch): the tile kernel instead
bool getenv_flag_off(const char* name) {
    const char* e = getenv(name);
    return !(e && e[0] == '0' && e[1] == 0);
}

bool f32_narrow_eligible(const ConvGemmParams& p) {
    const char* e = getenv("VP3D_F32_NARROW");  // 0: never, 2: at any M (measurement)
    const bool any_m = e && e[0] == '2';
    return p.N <= 64 && (p.M < 256 * BM || any_m) && !p.R && p.Ktap == p.K && p.K % 16 == 0 && p.K <= p.Kp &&
           p.lda % 4 == 0 && p.Kp % 4 == 0 && aligned(p.A, 16) && aligned(p.W, 16) && getenv_flag_off("VP3D_F32_NARROW");
}

bool narrow_eligible(const ConvGemmParams& p, Act a_type, Act out_type, Act compute) {
    // only while the 128-row tiles would leave CUs idle (< 256 tiles): B = 8192 windows
    // 0.036 -> 0.018 ms; at 65,536 rows the tile kernel stays ahead (0.048 vs 0.086 ms)
    return compute != Act::F32 && a_type == compute && out_type == Act::F32 && p.N <= 64 && p.M < 256 * BM &&
           p.Ktap == p.K &&
           p.K % 32 == 0 && p.Kp >= 64 && p.lda % 8 == 0 && aligned(p.A, 16) && !p.R;
}

}  // namespace

hipError_t launch_conv_gemm(const ConvGemmParams& p, Act a_type, Act out_type, Act compute,
                            hipStream_t stream) {
    if (p.M <= 0 || p.N <= 0) return hipSuccess;
    const int ntm = (p.M + BM - 1) / BM;
    const int ntn = (p.N + BN - 1) / BN;
    const dim3 grid(ntm * ntn);
    const bool contiguous = p.Ktap == p.K;  // taps collapsed into one K segment
    const int oes = out_type == Act::F32 ? 4 : 2;
    const bool vepi = (p.N % 8 == 0) && (p.ldy % 8 == 0) && aligned(p.Y, 16) &&
                      (!p.R || ((p.ldr % 8 == 0) && aligned(p.R, 16))) && oes > 0;
    if (compute == Act::F32) {
        if (a_type != Act::F32 || out_type != Act::F32) return hipErrorInvalidValue;
        if (f32_narrow_eligible(p)) {
            hipLaunchKernelGGL(conv_gemm_f32_narrow, dim3((p.M + 15) / 16), dim3(256), 0, stream, p);
            return hipGetLastError();
        }
        if ((p.Ktap % kF32Bk == 0) && (p.lda % 4 == 0) && aligned(p.A, 16))
            return launch_f32<A_VEC>(p, vepi, grid, stream);
        if (contiguous && (p.lda % 2 == 0) && (p.K % 2 == 0) && aligned(p.A, 8))
            return launch_f32<A_PAIRS>(p, vepi, grid, stream);
        return launch_f32<A_SCALAR>(p, vepi, grid, stream);
    }
    if (a_type != Act::F32 && a_type != compute) return hipErrorInvalidValue;
    if (out_type != Act::F32 && out_type != compute) return hipErrorInvalidValue;
    if (narrow_eligible(p, a_type, out_type, compute)) {
        const dim3 g((p.M + 15) / 16);
        if (compute == Act::BF16)
            hipLaunchKernelGGL(conv_gemm_narrow<bf16>, g, dim3(256), 0, stream, p);
        else
            hipLaunchKernelGGL(conv_gemm_narrow<f16>, g, dim3(256), 0, stream, p);
        return hipGetLastError();
    }
    const int gm = gemm_8p_mode();
    if ((gm == 5 || gm == 1) && conv_gemm_a4_eligible(p, a_type, out_type, compute) && conv_gemm_a4_fills(p))
        return launch_conv_gemm_a4(p, compute, stream);
    // q64 also below 384 tiles (round 5): it sums every output in a4's K order, so a layer gives
    // the same bits at every batch size (the 128 x 128 kernel's order differs: config 4's block-4
    // 1x1 at 8,192 windows per GPU broke bit identity across shard sizes)
    if ((gm == 3 || (gm == 1 && p.dil == 1)) && conv_gemm_q64_eligible(p, a_type, out_type, compute))
        return launch_conv_gemm_q64(p, compute, stream);
    if (gemm_8p_env(p) && conv_gemm_big_eligible(p, a_type, out_type, compute) &&
        conv_gemm_8p_eligible(p, a_type, out_type, compute))
        return launch_conv_gemm_8p(p, compute, stream);
    if (gm != 4 && conv_gemm_big_eligible(p, a_type, out_type, compute))
        return launch_conv_gemm_big(p, out_type, compute, stream);
    const int aes = a_type == Act::F32 ? 4 : 2;
    int amode = A_SCALAR;
    if ((p.Ktap % kH16Bk == 0) && (p.lda % 8 == 0) && aligned(p.A, 16))
        amode = A_VEC;
    else if (aes == 4 && contiguous && (p.lda % 2 == 0) && (p.K % 2 == 0) && aligned(p.A, 8))
        amode = A_PAIRS;
    if (compute == Act::BF16) return launch_h16_dispatch<bf16>(p, a_type, out_type, amode, vepi, grid, stream);
    return launch_h16_dispatch<f16>(p, a_type, out_type, amode, vepi, grid, stream);
}

}  // namespace vp3d
