// 256x256-tile conv-GEMM for the large 1024-channel layers (16-bit operands).
//
// Same contract as conv_gemm.hip (ConvGemmParams, kernels.h) restricted to the
// tap-aligned case (Ktap % 32 == 0, 16-bit activations): the block convolutions
// and 1x1 convolutions of TemporalModel / TemporalModelOptimized1f
// (reference common/models/TemporalModel.py:113-119, :179-181).
//
// Why a second family: at 128x128 the operand stream (32 KB per 2.1 MFLOP K-step)
// saturates the L2 (~34 TB/s chip-wide) well below the MFMA peak; a 256x256 tile
// moves 32 KB per 4.2 MFLOP K-step of 32.
//
// Structure (one 512-thread workgroup per CU, 8 waves as 2(M) x 4(N), each wave a
// 128x64 sub-tile = 8x4 v_mfma_f32_16x16x32_{bf16,f16} blocks):
//   * operands move HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4): no VGPR
//     staging, 4 DMA instructions per wave per K-step;
//   * a 4-slot ring of 32-deep K-steps (4 x 32 KB = 128 KB of LDS): while slot s is
//     consumed, slots s+1..s+3 are in flight; one counted `s_waitcnt vmcnt` + one
//     raw s_barrier per K-step (never vmcnt(0) inside the loop);
//   * LDS rows are 64 B (32 elements); the 16-byte chunk c of row r is stored at
//     chunk (c + 2*((r>>2)&3)) & 3, which makes every ds_read_b128 fragment read
//     bank-conflict free; LDS-DMA writes lane-linear, so the swizzle is applied to
//     each lane's SOURCE address (its inverse permutation), never to the LDS side;
//   * the workgroup -> tile map is XCD-aware (consecutive tiles on one XCD share
//     the A panel in that XCD's L2).
#include <cstdlib>
#include <cstring>

#include "gemm_common.h"

namespace vp3d {
namespace {

using namespace gemm;

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int BM2 = 256;
constexpr int BK2 = 32;

template <int NW_N, int NSLOT>
struct BigCfg {
    static constexpr int BN = 64 * NW_N;                 // 256 (8 waves) or 128 (4 waves)
    static constexpr int NWAVES = 2 * NW_N;
    static constexpr int THREADS = 64 * NWAVES;
    static constexpr int A_PIECES = (BM2 / 16) / NWAVES;  // 1 KB LDS-DMA pieces per wave per K-step
    static constexpr int B_PIECES = (BN / 16) / NWAVES;
    static constexpr int DMA_PER_STEP = A_PIECES + B_PIECES;
    static constexpr int SLOT_BYTES = (BM2 + BN) * BK2 * 2;
    static constexpr int RING_BYTES = NSLOT * SLOT_BYTES;
    static constexpr int EPI_BYTES = NWAVES * 32 * kEpiLd * 4;
    static constexpr int SMEM = RING_BYTES > EPI_BYTES ? RING_BYTES : EPI_BYTES;
};

// Counted wait: this wave's LDS-DMA of the current K-step has landed while `after`
// later K-steps (DMA_PER_STEP instructions each) stay in flight.
template <int PER_STEP>
__device__ __forceinline__ void wait_vm(int after) {
    if (after >= 3)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER_STEP) : "memory");
    else if (after == 2)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER_STEP) : "memory");
    else if (after == 1)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_STEP) : "memory");
    else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void block_sync_lds() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Main loop (one schedule; round 1 measured plain / prio / spread variants at
// 1010-1130 TFLOP/s vs 1138 for this one on the block-1 k3 layer): the fragments of
// K-step s+1 are read from LDS into a second register set while the MFMAs of step s
// run, and the program order is pinned with sched_barrier: per group g of 4 MFMAs
// (A row g), two (g < 6) fragment reads of the next step and one LDS-DMA refill piece.
template <typename CT, typename OT>
__global__ __launch_bounds__(512, 2) void conv_gemm_h16_big(ConvGemmParams p) {
    using C = BigCfg<4, 4>;
    constexpr int NSLOT = 4;
    __shared__ __attribute__((aligned(16))) char smem[C::SMEM];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wr = wid / 4, wc = wid % 4;

    const int ntn = (p.N + C::BN - 1) / C::BN;
    const int ntm = (p.M + BM2 - 1) / BM2;
    const int wg = xcd_remap(blockIdx.x, ntm * ntn);
    const int tile_m = wg / ntn;
    const int tile_n = wg - tile_m * ntn;
    const int m0 = tile_m * BM2, n0 = tile_n * C::BN;

    // ---- LDS-DMA source addressing (per lane, fixed for the whole K loop) ----
    // Piece pc of an operand covers rows pc*16 .. pc*16+15 (1 KB); wave w issues
    // pieces w, w + NWAVES, ...  Lane l fills LDS chunk (l & 3) of row
    // pc*16 + (l >> 2); that physical chunk holds logical chunk dma_c:
    const int dma_row = lane >> 2;
    const int dma_c = ((lane & 3) - 2 * ((lane >> 4) & 3)) & 3;
    int a_src[C::A_PIECES];
    int64_t b_off[C::B_PIECES];
#pragma unroll
    for (int q = 0; q < C::A_PIECES; ++q) {
        int m = m0 + (wid + C::NWAVES * q) * 16 + dma_row;
        m = m < p.M ? m : p.M - 1;  // rows past M read a valid row; their outputs are never stored
        a_src[q] = src_row(p, m);
    }
#pragma unroll
    for (int q = 0; q < C::B_PIECES; ++q) {
        const int n = n0 + (wid + C::NWAVES * q) * 16 + dma_row;  // W rows padded to 256
        b_off[q] = (int64_t)n * p.Kp + dma_c * 8;
    }
    const CT* A = (const CT*)p.A;
    const CT* W = (const CT*)p.W;

    // one LDS-DMA piece of K-step s: idx < A_PIECES -> A piece, else B piece
    auto issue_piece = [&](int s, int idx) {
        const int k0 = s * BK2;
        char* slot = smem + (s % NSLOT) * C::SLOT_BYTES;
        if (idx < C::A_PIECES) {
            const int tap = k0 / p.Ktap;
            const int cin = k0 - tap * p.Ktap + dma_c * 8;
            const CT* ga = A + (int64_t)(a_src[idx] + tap * p.dil) * p.lda + cin;
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)ga,
                                             (lds_ptr_t)(slot + (wid + C::NWAVES * idx) * 1024), 16, 0, 0);
        } else {
            const int q = idx - C::A_PIECES;
            const CT* gb = W + b_off[q] + k0;
            __builtin_amdgcn_global_load_lds(
                (gbl_ptr_t)gb, (lds_ptr_t)(slot + BM2 * BK2 * 2 + (wid + C::NWAVES * q) * 1024), 16, 0, 0);
        }
    };
    auto issue = [&](int s) {
#pragma unroll
        for (int idx = 0; idx < C::DMA_PER_STEP; ++idx) issue_piece(s, idx);
    };

    // ---- fragment reads: row (l & 15) of each 16-row block, logical chunk (l >> 4)
    // -> physical chunk (c + 2*((r>>2)&3)) & 3, lane-constant ----
    const int frag_chunk = ((lane >> 4) + 2 * (((lane & 15) >> 2) & 3)) & 3;
    const int a_frag_off = (wr * 128 + (lane & 15)) * 64 + frag_chunk * 16;
    const int b_frag_off = BM2 * BK2 * 2 + (wc * 64 + (lane & 15)) * 64 + frag_chunk * 16;

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    struct Frag {
        u32x4 a[8];
        u32x4 b[4];
    };
    auto read_frags = [&](int s, Frag& f) {
        const char* slot = smem + (s % NSLOT) * C::SLOT_BYTES;
#pragma unroll
        for (int j = 0; j < 4; ++j) f.b[j] = *(const u32x4*)(slot + b_frag_off + j * 16 * 64);
#pragma unroll
        for (int i = 0; i < 8; ++i) f.a[i] = *(const u32x4*)(slot + a_frag_off + i * 16 * 64);
    };
    auto mma = [&](const Frag& f) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma16<CT>(f.a[i], f.b[j], acc[i][j]);
    };

    const int nk = p.Kp / BK2;
    const int pre = nk < NSLOT - 1 ? nk : NSLOT - 1;
    for (int s = 0; s < pre; ++s) issue(s);

    // stage s+1 must be resident one step early; slot s-1 (read during step s-2,
    // consumed by step s-1) is the one refilled at step s
    wait_vm<C::DMA_PER_STEP>(pre - 1);
    block_sync_lds();
    Frag f0, f1;
    read_frags(0, f0);
    // steady state: compile-time wait counts, no branches between the reads and the MFMAs
    auto step_full = [&](int s, Frag& cur, Frag& nxt) {
        wait_vm<C::DMA_PER_STEP>(NSLOT - 3);
        block_sync_lds();
        const char* slot = smem + ((s + 1) % NSLOT) * C::SLOT_BYTES;
#pragma unroll
        for (int g = 0; g < 8; ++g) {
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[g][j] = mfma16<CT>(cur.a[g], cur.b[j], acc[g][j]);
            __builtin_amdgcn_sched_barrier(0);
            if (g < 2) {
                nxt.b[2 * g] = *(const u32x4*)(slot + b_frag_off + (2 * g) * 16 * 64);
                nxt.b[2 * g + 1] = *(const u32x4*)(slot + b_frag_off + (2 * g + 1) * 16 * 64);
            } else if (g < 6) {
                nxt.a[2 * (g - 2)] = *(const u32x4*)(slot + a_frag_off + (2 * (g - 2)) * 16 * 64);
                nxt.a[2 * (g - 2) + 1] = *(const u32x4*)(slot + a_frag_off + (2 * (g - 2) + 1) * 16 * 64);
            }
            if (g < C::DMA_PER_STEP) issue_piece(s + NSLOT - 1, g);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    int s = 0;
    for (; s + NSLOT < nk; s += 2) {
        step_full(s, f0, f1);
        step_full(s + 1, f1, f0);
    }
    // tail: the last few steps (no refills, runtime wait counts)
    auto step_tail = [&](int s2, Frag& cur, Frag& nxt) {
        if (s2 + 1 < nk) {
            const int issued = nk < s2 + NSLOT - 1 ? nk : s2 + NSLOT - 1;
            wait_vm<C::DMA_PER_STEP>(issued - (s2 + 2));
            block_sync_lds();
            if (s2 + NSLOT - 1 < nk) issue(s2 + NSLOT - 1);
        }
        read_frags(s2 + 1, nxt);  // past the last step this reads a stale slot, unused
        mma(cur);
    };
    for (; s < nk; s += 2) {
        step_tail(s, f0, f1);
        if (s + 1 < nk) step_tail(s + 1, f1, f0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    const int mw = m0 + wr * 128, nw = n0 + wc * 64;
    epilogue_vec<OT, 8, 32>(p, acc, (float*)smem + wid * 32 * kEpiLd, mw, nw, lane);
}

}  // namespace

bool conv_gemm_big_eligible(const ConvGemmParams& p, Act a_type, Act out_type, Act compute) {
    if (compute == Act::F32 || a_type != compute) return false;
    if (out_type != Act::F32 && out_type != compute) return false;
    if (p.Ktap % BK2 != 0 || p.Kp % BK2 != 0 || p.lda % 8 != 0) return false;
    if (p.N % 8 != 0 || p.ldy % 8 != 0 || (p.R && p.ldr % 8 != 0)) return false;
    if ((reinterpret_cast<uintptr_t>(p.A) & 15) || (reinterpret_cast<uintptr_t>(p.Y) & 15) ||
        (p.R && (reinterpret_cast<uintptr_t>(p.R) & 15)))
        return false;
    // enough tiles to fill the 256 CUs (block 3 of the 1f model at B = 8192: 384 tiles,
    // 1.5 rounds, still ahead of the 128x128 kernel: 0.17 vs 0.21 ms)
    const int64_t tiles = (int64_t)((p.M + BM2 - 1) / BM2) * ((p.N + 255) / 256);
    return tiles >= 384;
}

template <typename CT, typename OT>
hipError_t launch_big_t(const ConvGemmParams& p, hipStream_t stream) {
    const dim3 g(((p.M + BM2 - 1) / BM2) * ((p.N + 255) / 256));
    hipLaunchKernelGGL((conv_gemm_h16_big<CT, OT>), g, dim3(512), 0, stream, p);
    return hipGetLastError();
}

hipError_t launch_conv_gemm_big(const ConvGemmParams& p, Act out_type, Act compute,
                                hipStream_t stream) {
    if (compute == Act::BF16)
        return out_type == Act::F32 ? launch_big_t<bf16, float>(p, stream)
                                    : launch_big_t<bf16, bf16>(p, stream);
    return out_type == Act::F32 ? launch_big_t<f16, float>(p, stream)
                                : launch_big_t<f16, f16>(p, stream);
}

}  // namespace vp3d
