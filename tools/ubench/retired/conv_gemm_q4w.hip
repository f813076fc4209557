// RETIRED (not built): measured on MI355X (gpurun_out r03g, B = 65,536 bf16): bit-identical
// output, block-1 k3 40.2 ms vs 9.2 ms on conv_gemm_q64, every q64 layer 3.3-3.9x slower.  At
// one wave per SIMD the 256 AGPR accumulators plus two fragment sets leave the compiler 201
// VGPR spills (the LDS address registers reloaded from scratch inside the K loop).
// 256x256 conv-GEMM at ONE wave per SIMD: 4 waves, each owning a 128 x 128 output tile
// (16-bit operands, 16-bit output).
//
// Contract: that of conv_gemm_q64 (ConvGemmParams, kernels.h): tap-aligned 16-bit
// activations (Ktap % 64 == 0), N % 256 == 0 -- the block k-convs and 1x1 convs of
// TemporalModel / TemporalModelOptimized1f (reference common/models/TemporalModel.py:113-119,
// :129-135, :179-181, :191-195).
//
// Why: q64 runs 8 waves of 128 x 64, two per SIMD; per 64-deep K-tile a CU reads 192 KiB of
// fragments from LDS and lands 64 KiB of LDS-DMA -- about as many LDS cycles as MFMA
// cycles.  A 128 x 128 wave tile reads 32 KiB per K-tile (128 KiB per CU, a third less
// per MFMA); the single wave on a SIMD keeps its MFMA stream busy by itself: fragments are
// double-buffered in registers (two sets of 8 A + 8 W fragments), so the reads of the next
// half K-tile are in flight under the MFMAs of the current one, with ONE barrier per K-tile.
// The 256 accumulators per lane live in AGPRs (the MFMAs are inline asm with "+a" operands:
// left to itself the register allocator shuffles them between AGPRs and VGPRs inside the
// loop, ~200 v_accvgpr moves per K-tile).
//
// K-tile t (64 deep, LDS buffer t & 1, staged by LDS-DMA as whole 128-byte lines with
// q64's chunk swizzle):
//   phase A: 64 MFMAs on fragment set 0 (k 0..31 of tile t), reads of set 1 (k 32..63 of t)
//   mid:     vmcnt(0) (tile t + 1 landed: this wave's pieces), lgkmcnt(0) (tile t read out
//            by this wave), barrier; then this wave's DMA pieces of tile t + 2 into buffer
//            t & 1, which every wave has finished reading
//   phase B: 64 MFMAs on set 1, reads of set 0 (k 0..31 of tile t + 1)
// Epilogue: gemm::epilogue_tp, twice (64 channels each).
#include "gemm_common.h"

namespace vp3d {
namespace {

using namespace gemm;

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int WM = 256, WN = 256, WK = 64;
constexpr int WBUF = (WM + WN) * WK * 2;  // 64 KiB per buffer
constexpr int WW_OFF = WM * WK * 2;       // W region inside a buffer
constexpr int WMAXN = 1024;

__device__ __forceinline__ void pinned_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

// D = W . A^T + D with the accumulator pinned to AGPRs
template <typename CT>
__device__ __forceinline__ void mfma_a(f32x4& acc, const u32x4& w, const u32x4& a);
template <>
__device__ __forceinline__ void mfma_a<__bf16>(f32x4& acc, const u32x4& w, const u32x4& a) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(w), "v"(a));
}
template <>
__device__ __forceinline__ void mfma_a<_Float16>(f32x4& acc, const u32x4& w, const u32x4& a) {
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(w), "v"(a));
}

template <typename CT>
__global__ __launch_bounds__(256, 1) void conv_gemm_q4w(ConvGemmParams p) {
    __shared__ __attribute__((aligned(16))) char smem[2 * WBUF + 2 * WMAXN * 4];
    float* const s_scale = (float*)(smem + 2 * WBUF);
    float* const s_shift = s_scale + WMAXN;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wr = wid >> 1, wc = wid & 1;

    for (int i = tid; i < p.N; i += 256) {
        s_scale[i] = p.scale[i];
        s_shift[i] = p.shift[i];
    }

    const int ntn = p.N / WN;
    const int ntm = (p.M + WM - 1) / WM;
    const int wg = xcd_remap(blockIdx.x, ntm * ntn);
    const int tile_m = wg / ntn;
    const int tile_n = wg - tile_m * ntn;
    const int m0 = tile_m * WM, n0 = tile_n * WN;

    // ---- DMA pieces: 8 rows x 128 B each, 32 per operand; wave w issues q = w + 4 i ----
    const int prow = lane >> 3;
    // all pieces of a wave share the parity of q (= that of w): one swizzled chunk each
    const int lc = (lane & 7) ^ (((wid & 1) * 4 + (prow >> 1)) & 7);
    int a_src[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        int m = m0 + 8 * (wid + 4 * i) + prow;
        m = m < p.M ? m : p.M - 1;  // rows past M read a valid row; never stored
        a_src[i] = src_row(p, m);
    }
    const int w_off0 = (n0 + 8 * wid + prow) * p.Kp + lc * 8;  // piece i: + 32 i rows
    const CT* A = (const CT*)p.A;
    const CT* W = (const CT*)p.W;
    auto issue_tile = [&](int s) {
        char* buf = smem + (s & 1) * WBUF;
        const int k0 = s * WK;
        const int tap = k0 / p.Ktap;
        const int cb = k0 - tap * p.Ktap;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            __builtin_amdgcn_global_load_lds(
                (gbl_ptr_t)(A + (int64_t)(a_src[i] + tap * p.dil) * p.lda + cb + lc * 8),
                (lds_ptr_t)(buf + (wid + 4 * i) * 1024), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(W + w_off0 + 32 * i * p.Kp + k0),
                                             (lds_ptr_t)(buf + WW_OFF + (wid + 4 * i) * 1024), 16, 0, 0);
    };

    // ---- fragment reads (q64's layout): row (l & 15) of a 16-row block, logical chunk
    // 4 kh + (l >> 4), physical chunk ^ ((l & 15) >> 1) ----
    const int fsw = (lane & 15) >> 1;
    const int fo0 = (lane & 15) * 128 + (((lane >> 4) ^ fsw) << 4);
    const int fo1 = (lane & 15) * 128 + ((((lane >> 4) + 4) ^ fsw) << 4);
    const int a_base = wr * 128 * 128;
    const int w_base = WW_OFF + wc * 128 * 128;

    f32x4 acc[2][8][4];  // [channel half][row block][channel block]
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // fragment sets [set][block]; the reads are inline asm too, placed between the MFMAs
    // in program order (one A and one W read per row block of MFMAs), with the lgkmcnt
    // waits written out: the compiler neither hoists them into a burst nor waits early
    u32x4 fa[2][8], fw[2][8];
    // LDS byte addresses of the fragment rows: [buffer][kh] (A, W); block i at + 2048 i
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    uint32_t ad_a[2][2], ad_w[2][2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        ad_a[b][0] = lds0 + b * WBUF + a_base + fo0;
        ad_a[b][1] = lds0 + b * WBUF + a_base + fo1;
        ad_w[b][0] = lds0 + b * WBUF + w_base + fo0;
        ad_w[b][1] = lds0 + b * WBUF + w_base + fo1;
    }
#define Q4W_RD(dst, addr, blk) \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "i"((blk) * 2048))
    // 64 MFMAs on set `cur`, the 16 reads of set `nxt` from (buffer b, kh) spread among them
    auto phase = [&](int cur, int nxt, bool rd, int b, int kh) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (rd) {  // (always: kept as a parameter for measurement builds)
                switch (i) {  // constant block index for the immediate offset
                    case 0: Q4W_RD(fa[nxt][0], ad_a[b][kh], 0); Q4W_RD(fw[nxt][0], ad_w[b][kh], 0); break;
                    case 1: Q4W_RD(fa[nxt][1], ad_a[b][kh], 1); Q4W_RD(fw[nxt][1], ad_w[b][kh], 1); break;
                    case 2: Q4W_RD(fa[nxt][2], ad_a[b][kh], 2); Q4W_RD(fw[nxt][2], ad_w[b][kh], 2); break;
                    case 3: Q4W_RD(fa[nxt][3], ad_a[b][kh], 3); Q4W_RD(fw[nxt][3], ad_w[b][kh], 3); break;
                    case 4: Q4W_RD(fa[nxt][4], ad_a[b][kh], 4); Q4W_RD(fw[nxt][4], ad_w[b][kh], 4); break;
                    case 5: Q4W_RD(fa[nxt][5], ad_a[b][kh], 5); Q4W_RD(fw[nxt][5], ad_w[b][kh], 5); break;
                    case 6: Q4W_RD(fa[nxt][6], ad_a[b][kh], 6); Q4W_RD(fw[nxt][6], ad_w[b][kh], 6); break;
                    default: Q4W_RD(fa[nxt][7], ad_a[b][kh], 7); Q4W_RD(fw[nxt][7], ad_w[b][kh], 7); break;
                }
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) mfma_a<CT>(acc[j >> 2][i][j & 3], fw[cur][j], fa[cur][i]);
        }
    };

    const int nk = p.Kp / WK;
    issue_tile(0);
    if (nk > 1) issue_tile(1);
    if (nk > 1)
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 0 landed (younger: tile 1)
    else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // scale / shift stores
    pinned_barrier();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        fa[0][i] = *(const u32x4*)(smem + a_base + i * 16 * 128 + fo0);
        fw[0][i] = *(const u32x4*)(smem + w_base + i * 16 * 128 + fo0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

    // two K-tiles per trip, so the LDS buffer of each phase is a compile-time constant; the
    // last phase B reads (unused) fragments of the other buffer instead of branching
    auto ktile = [&](int t, int b) {
        // ---- phase A: set 0 (k 0..31 of t) under the reads of set 1 (k 32..63 of t) ----
        phase(0, 1, true, b, 1);
        // ---- mid: tile t + 1 landed, tile t read out; stage tile t + 2 into t's buffer ----
        asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
        pinned_barrier();
        if (t + 2 < nk) issue_tile(t + 2);
        asm volatile("" ::: "memory");
        // ---- phase B: set 1 under the reads of set 0 (k 0..31 of t + 1) ----
        phase(1, 0, true, b ^ 1, 0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    for (int t = 0; t < nk; t += 2) {
        ktile(t, 0);
        if (t + 1 < nk) ktile(t + 1, 1);
    }
#undef Q4W_RD
    // the last MFMAs' results: MFMA -> VALU read of the accumulator (inline-asm MFMAs are
    // not tracked by the compiler's hazard recognizer)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

    const size_t y_rest = (size_t)(p.M - m0) * p.ldy * sizeof(CT);
    const __amdgpu_buffer_rsrc_t y_rsrc =
        make_rsrc((const CT*)p.Y + (size_t)m0 * p.ldy, (uint32_t)(y_rest < 0x7FFFFFFFu ? y_rest : 0x7FFFFFFFu));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (p.R)
            epilogue_tp<CT, 8, false, 1, 0>(p, acc[h], m0 + wr * 128, n0 + wc * 128 + 64 * h, lane, s_scale, s_shift,
                                            y_rsrc, nullptr, m0);
        else
            epilogue_tp<CT, 8, false, 0, 0>(p, acc[h], m0 + wr * 128, n0 + wc * 128 + 64 * h, lane, s_scale, s_shift,
                                            y_rsrc, nullptr, m0);
    }
}

}  // namespace

hipError_t launch_conv_gemm_q4w(const ConvGemmParams& p, Act compute, hipStream_t stream) {
    const dim3 grid(((p.M + WM - 1) / WM) * (p.N / WN));
    if (compute == Act::BF16)
        hipLaunchKernelGGL((conv_gemm_q4w<__bf16>), grid, dim3(256), 0, stream, p);
    else
        hipLaunchKernelGGL((conv_gemm_q4w<_Float16>), grid, dim3(256), 0, stream, p);
    return hipGetLastError();
}

}  // namespace vp3d
