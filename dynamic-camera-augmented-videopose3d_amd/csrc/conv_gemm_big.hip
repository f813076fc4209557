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
#include "gemm_common.h"

namespace vp3d {
namespace {

using namespace gemm;

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int BM2 = 256;
constexpr int BN2 = 256;
constexpr int BK2 = 32;
constexpr int NSLOT = 4;
constexpr int SLOT_BYTES = (BM2 + BN2) * BK2 * 2;  // 32 KB: A rows then B rows
constexpr int RING_BYTES = NSLOT * SLOT_BYTES;     // 128 KB
constexpr int EPI_BYTES = 8 * 32 * kEpiLd * 4;     // 8 waves x 32-row passes
constexpr int SMEM2 = RING_BYTES > EPI_BYTES ? RING_BYTES : EPI_BYTES;

__device__ __forceinline__ void wait_vm(int n_after) {
    // outstanding LDS-DMA of this wave allowed to remain in flight (4 per K-step)
    if (n_after >= 2)
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n_after == 1)
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void block_sync_lds() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <typename CT, typename OT>
__global__ __launch_bounds__(512, 2) void conv_gemm_h16_256(ConvGemmParams p) {
    __shared__ __attribute__((aligned(16))) char smem[SMEM2];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wr = wid >> 2, wc = wid & 3;

    const int ntn = (p.N + BN2 - 1) / BN2;
    const int ntm = (p.M + BM2 - 1) / BM2;
    const int wg = xcd_remap(blockIdx.x, ntm * ntn);
    const int tile_m = wg / ntn;
    const int tile_n = wg - tile_m * ntn;
    const int m0 = tile_m * BM2, n0 = tile_n * BN2;

    // ---- LDS-DMA source addressing (per lane, fixed for the whole K loop) ----
    // A wave issues pieces {wid, wid+8} of A and of B per K-step; piece pc covers
    // rows pc*16 .. pc*16+15 (1 KB).  Lane l fills LDS chunk (l & 3) of row
    // pc*16 + (l >> 2); that physical chunk holds logical chunk c:
    const int dma_row = lane >> 2;
    const int dma_c = ((lane & 3) - 2 * ((lane >> 4) & 3)) & 3;
    int a_src[2];
    int64_t b_off[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int pc = wid + 8 * q;
        int m = m0 + pc * 16 + dma_row;
        m = m < p.M ? m : p.M - 1;  // rows past M read a valid row; their outputs are never stored
        a_src[q] = src_row(p, m);
        const int n = n0 + pc * 16 + dma_row;  // W is padded to a multiple of 256 rows
        b_off[q] = (int64_t)n * p.Kp + dma_c * 8;
    }
    const CT* A = (const CT*)p.A;
    const CT* W = (const CT*)p.W;

    auto issue = [&](int s) {
        const int k0 = s * BK2;
        const int tap = k0 / p.Ktap;
        const int cin = k0 - tap * p.Ktap + dma_c * 8;
        char* slot = smem + (s % NSLOT) * SLOT_BYTES;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int pc = wid + 8 * q;
            const CT* ga = A + (int64_t)(a_src[q] + tap * p.dil) * p.lda + cin;
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)ga, (lds_ptr_t)(slot + pc * 1024), 16, 0, 0);
            const CT* gb = W + b_off[q] + k0;
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)gb,
                                             (lds_ptr_t)(slot + BM2 * BK2 * 2 + pc * 1024), 16, 0, 0);
        }
    };

    // ---- fragment read addressing: row (l & 15) of each 16-row block, logical
    // chunk (l >> 4) -> physical chunk (c + 2*((r>>2)&3)) & 3 (lane-constant) ----
    const int frag_chunk = ((lane >> 4) + 2 * (((lane & 15) >> 2) & 3)) & 3;
    const int a_frag_off = (wr * 128 + (lane & 15)) * 64 + frag_chunk * 16;
    const int b_frag_off = BM2 * BK2 * 2 + (wc * 64 + (lane & 15)) * 64 + frag_chunk * 16;

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = p.Kp / BK2;
    const int pre = nk < NSLOT - 1 ? nk : NSLOT - 1;
    for (int s = 0; s < pre; ++s) issue(s);

    for (int s = 0; s < nk; ++s) {
        const int left = nk - 1 - s;  // K-steps after s already issued (capped at 2)
        wait_vm(left < 2 ? left : 2);
        block_sync_lds();  // slot s landed for every wave; slot s-1 fully consumed
        if (s + NSLOT - 1 < nk) issue(s + NSLOT - 1);
        const char* slot = smem + (s % NSLOT) * SLOT_BYTES;
        u32x4 bfr[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = *(const u32x4*)(slot + b_frag_off + j * 16 * 64);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const u32x4 afr = *(const u32x4*)(slot + a_frag_off + i * 16 * 64);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma16<CT>(afr, bfr[j], acc[i][j]);
        }
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
    // enough tiles to fill the 256 CUs about four times over
    const int64_t tiles = (int64_t)((p.M + BM2 - 1) / BM2) * ((p.N + BN2 - 1) / BN2);
    return tiles >= 4 * 256;
}

hipError_t launch_conv_gemm_big(const ConvGemmParams& p, Act out_type, Act compute,
                                hipStream_t stream) {
    const dim3 grid(((p.M + BM2 - 1) / BM2) * ((p.N + BN2 - 1) / BN2));
    if (compute == Act::BF16) {
        if (out_type == Act::F32)
            hipLaunchKernelGGL((conv_gemm_h16_256<bf16, float>), grid, dim3(512), 0, stream, p);
        else
            hipLaunchKernelGGL((conv_gemm_h16_256<bf16, bf16>), grid, dim3(512), 0, stream, p);
    } else {
        if (out_type == Act::F32)
            hipLaunchKernelGGL((conv_gemm_h16_256<f16, float>), grid, dim3(512), 0, stream, p);
        else
            hipLaunchKernelGGL((conv_gemm_h16_256<f16, f16>), grid, dim3(512), 0, stream, p);
    }
    return hipGetLastError();
}

}  // namespace vp3d
