// Ping-pong 256x256 conv-GEMM: the two wave groups of the workgroup run one
// barrier apart, so on every SIMD one wave issues its 16 MFMAs while the other
// issues its LDS fragment reads and LDS-DMA pieces.
//
// Same contract as conv_gemm_big.hip (ConvGemmParams, tap-aligned 16-bit
// activations; reference common/models/TemporalModel.py:113-119, :179-181), same
// LDS image (4-slot ring of 32-deep K-steps, 64-B rows, chunk swizzle on the DMA
// source) and the same 2(M) x 4(N) wave grid with 128x64 per wave.  What differs
// is the schedule:
//   * a K-step is two phases; phase h of step s reads A blocks 4h..4h+3 (and, in
//     phase 0, the 4 B blocks) of slot s, then, behind a barrier, runs the 16
//     MFMAs acc[4h+i][j] at raised priority, then a second barrier;
//   * group 1 (wr == 1) enters one barrier late and group 0 leaves one barrier
//     late, so group 0's MFMA part coincides with group 1's read part and vice
//     versa (cdna_hip_programming.md §5, the 256^2 8-phase template's stagger);
//   * each wave owns 4 LDS-DMA pieces per K-step (2 of A, 2 of B).  Refill of
//     step s+3 (the slot step s-1 used) is issued by group 1 in both phases of
//     step s and by group 0 in phase 1 of step s and phase 0 of step s+1: both
//     are past the barrier that retires every read of step s-1 (WAR);
//   * in phase 0 of step s each wave waits (counted vmcnt) for its pieces of
//     step s+1, which is read two barriers later (RAW).
#include <cstdlib>

#include "gemm_common.h"

namespace vp3d {
namespace {

using namespace gemm;

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int QM = 256, QN = 256, QK = 32;
constexpr int QSLOTS = 4;
constexpr int QSLOT_BYTES = (QM + QN) * QK * 2;  // 32 KiB
constexpr int QRING = QSLOTS * QSLOT_BYTES;      // 128 KiB (epilogue staging reuses it)

__device__ __forceinline__ void bar() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void vmw() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <typename CT, typename OT>
__global__ __launch_bounds__(512) void conv_gemm_h16_pp(ConvGemmParams p) {
    __shared__ __attribute__((aligned(16))) char smem[QRING];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches
    const int wr = wid >> 2, wc = wid & 3;

    const int ntn = (p.N + QN - 1) / QN;
    const int ntm = (p.M + QM - 1) / QM;
    const int wg = xcd_remap(blockIdx.x, ntm * ntn);
    const int tile_m = wg / ntn;
    const int m0 = tile_m * QM, n0 = (wg - tile_m * ntn) * QN;

    // LDS-DMA: piece q of A covers rows (wid + 8q)*16 .. +15, lane l fills physical
    // chunk (l & 3) of row (l >> 2), which holds logical chunk dma_c.
    const int dma_row = lane >> 2;
    const int dma_c = ((lane & 3) - 2 * ((lane >> 4) & 3)) & 3;
    int a_src[2];
    int64_t b_off[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        int m = m0 + (wid + 8 * q) * 16 + dma_row;
        m = m < p.M ? m : p.M - 1;  // rows past M read a valid row; never stored
        a_src[q] = src_row(p, m);
        b_off[q] = (int64_t)(n0 + (wid + 8 * q) * 16 + dma_row) * p.Kp + dma_c * 8;  // W rows padded
    }
    const CT* A = (const CT*)p.A;
    const CT* W = (const CT*)p.W;
    // pieces 0,1: A; 2,3: B of K-step s
    auto dma2 = [&](int s, int first) {
        const int k0 = s * QK;
        char* slot = smem + (s % QSLOTS) * QSLOT_BYTES;
        if (first == 0) {
            const int tap = k0 / p.Ktap;
            const int cin = k0 - tap * p.Ktap + dma_c * 8;
#pragma unroll
            for (int q = 0; q < 2; ++q)
                __builtin_amdgcn_global_load_lds(
                    (gbl_ptr_t)(A + (int64_t)(a_src[q] + tap * p.dil) * p.lda + cin),
                    (lds_ptr_t)(slot + (wid + 8 * q) * 1024), 16, 0, 0);
        } else {
#pragma unroll
            for (int q = 0; q < 2; ++q)
                __builtin_amdgcn_global_load_lds((gbl_ptr_t)(W + b_off[q] + k0),
                                                 (lds_ptr_t)(slot + QM * QK * 2 + (wid + 8 * q) * 1024),
                                                 16, 0, 0);
        }
    };

    const int frag_chunk = ((lane >> 4) + 2 * (((lane & 15) >> 2) & 3)) & 3;
    const int a_frag_off = (wr * 128 + (lane & 15)) * 64 + frag_chunk * 16;
    const int b_frag_off = QM * QK * 2 + (wc * 64 + (lane & 15)) * 64 + frag_chunk * 16;

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = p.Kp / QK;
    const bool g1 = wr == 1;

    // ---- prologue: steps 0..2 in flight, step 0 landed ----
    for (int s = 0; s < 3 && s < nk; ++s) {
        dma2(s, 0);
        dma2(s, 1);
    }
    if (nk >= 3)
        vmw<8>();
    else if (nk == 2)
        vmw<4>();
    else
        vmw<0>();
    bar();
    if (g1) bar();  // stagger: group 1 runs one barrier behind

    u32x4 a[4], b[4];
    for (int s = 0; s < nk; ++s) {
        const char* slot = smem + (s % QSLOTS) * QSLOT_BYTES;
        // ---------- phase 0 ----------
        // own pieces of step s+1 landed; younger in flight: group 0 the A half of
        // step s+2 (the whole step at s == 0, from the prologue), group 1 all of s+2
        if (s + 2 < nk) {
            if (g1 || s == 0)
                vmw<4>();
            else
                vmw<2>();
        } else {
            vmw<0>();
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = *(const u32x4*)(slot + b_frag_off + j * 1024);
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = *(const u32x4*)(slot + a_frag_off + i * 1024);
        if (g1) {
            if (s + 3 < nk) dma2(s + 3, 0);
        } else {
            if (s >= 1 && s + 2 < nk) dma2(s + 2, 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        bar();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma16<CT>(a[i], b[j], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        bar();
        // ---------- phase 1 ----------
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = *(const u32x4*)(slot + a_frag_off + (4 + i) * 1024);
        if (s + 3 < nk) dma2(s + 3, g1 ? 1 : 0);
        __builtin_amdgcn_sched_barrier(0);
        bar();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[4 + i][j] = mfma16<CT>(a[i], b[j], acc[4 + i][j]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        bar();
    }
    if (!g1) bar();  // group 0 catches up: every read of the ring has retired
    vmw<0>();

    const int mw = m0 + wr * 128, nw = n0 + wc * 64;
    epilogue_vec<OT, 8, 32>(p, acc, (float*)smem + wid * 32 * kEpiLd, mw, nw, lane);
}

}  // namespace

hipError_t launch_conv_gemm_pp(const ConvGemmParams& p, Act out_type, Act compute, hipStream_t stream) {
    const dim3 grid(((p.M + QM - 1) / QM) * ((p.N + QN - 1) / QN));
    if (compute == Act::BF16) {
        if (out_type == Act::F32)
            hipLaunchKernelGGL((conv_gemm_h16_pp<__bf16, float>), grid, dim3(512), 0, stream, p);
        else
            hipLaunchKernelGGL((conv_gemm_h16_pp<__bf16, __bf16>), grid, dim3(512), 0, stream, p);
    } else {
        if (out_type == Act::F32)
            hipLaunchKernelGGL((conv_gemm_h16_pp<_Float16, float>), grid, dim3(512), 0, stream, p);
        else
            hipLaunchKernelGGL((conv_gemm_h16_pp<_Float16, _Float16>), grid, dim3(512), 0, stream, p);
    }
    return hipGetLastError();
}

}  // namespace vp3d
