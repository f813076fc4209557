// 256x256 conv-GEMM with a phase-split, wave-group ping-pong main loop and the
// register-direct epilogue (16-bit operands, 16-bit output).
//
// Contract: ConvGemmParams (kernels.h), tap-aligned 16-bit activations: the block
// convolutions and 1x1 convolutions of TemporalModel / TemporalModelOptimized1f
// (reference common/models/TemporalModel.py:113-119, :129-135, :179-181, :191-195).
//
// Geometry: 512 threads = 8 waves, wave (wr, wc) = (wid >> 2, wid & 3) owns output
// rows 128*wr .. +127 and channels 64*wc .. +63 of the tile.  Waves w and w+4 share a
// SIMD, so group G0 (wr = 0) and group G1 (wr = 1) put one wave on every SIMD.
// Operands: the LDS ring of conv_gemm_big.hip (4 slots of 32-deep K-steps, 32 KiB
// each, LDS-DMA with the swizzle applied to the source address).
//
// Main loop: each K-step s is two phases (rows 0-63 and 64-127 of the wave's rows),
// each phase = [memory segment: ds_reads of the phase's fragments + 2 LDS-DMA
// pieces] barrier, lgkmcnt(0), [16 v_mfma_f32_16x16x32 at s_setprio 1] barrier.
// G1 passes one extra barrier before the loop, so while G0 runs an MFMA segment
// G1 runs a memory segment and vice versa: the two waves of a SIMD alternate, and
// the MFMA pipe sees one wave's 16 MFMAs after the other's.
//   stage X's A pieces are issued in segment A of step X-2, its B pieces in
//   segment B of step X-3 (both into slots last read >= 3 barrier intervals earlier);
//   each wave waits (counted vmcnt, never 0 in steady state) for stage s+1 at the
//   end of segment B of step s, >= 1 barrier before any wave reads it.
// MFMA orientation D = W . A^T (weight fragment = A operand), so the epilogue is
// gemm::epilogue_tp: registers only, 16-byte buffer stores, no LDS.
#include <cstdlib>

#include "gemm_common.h"

namespace vp3d {
namespace {

using namespace gemm;

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int PM = 256, PN = 256, PK = 32;
constexpr int PSLOTS = 4;
constexpr int PSLOT_BYTES = (PM + PN) * PK * 2;  // 32 KiB
constexpr int PRING = PSLOTS * PSLOT_BYTES;      // 128 KiB
constexpr int PMAXN = 1024;

__device__ __forceinline__ void barrier_pinned() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void vmw() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ABL (ablation, measurement only): 0 = normal, 1 = no LDS-DMA inside the K loop
// (MFMA + LDS reads on stale data), 2 = no MFMAs (memory traffic only), 3 = no
// fragment reads after the first K-step (DMA + MFMA), 4 = neither reads nor DMA,
// 7 = normal + per-workgroup timestamps into g_trace (tools/ubench/gemm_check 8pt).
__device__ unsigned long long* g_trace;

__device__ __forceinline__ void trace_stamp(int wg, int slot) {
    // 100 MHz wall clock (comparable across CUs)
    const unsigned long long rt = __builtin_amdgcn_s_memrealtime();
    if (!g_trace) return;
    g_trace[(size_t)wg * 10 + slot] = rt;
}
template <typename CT, int ABL = 0>
__global__ __launch_bounds__(512, 1) void conv_gemm_8p(ConvGemmParams p) {
    __shared__ __attribute__((aligned(16))) char smem[PRING + 2 * PMAXN * 4];
    float* const s_scale = (float*)(smem + PRING);
    float* const s_shift = s_scale + PMAXN;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wr = wid >> 2, wc = wid & 3;

    for (int i = tid; i < p.N; i += 512) {
        s_scale[i] = p.scale[i];
        s_shift[i] = p.shift[i];
    }

    const int ntn = p.N / PN;
    const int ntm = (p.M + PM - 1) / PM;
    const int wg = xcd_remap(blockIdx.x, ntm * ntn);
    const int tile_m = wg / ntn;
    const int tile_n = wg - tile_m * ntn;
    const int m0 = tile_m * PM, n0 = tile_n * PN;
    if (ABL == 7 && tid == 0 && g_trace) {
        trace_stamp(blockIdx.x, 0);
        // slot 4: hardware ids (HW_ID: cu / sh / se; XCC_ID)
        g_trace[(size_t)blockIdx.x * 10 + 4] =
            ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
            __builtin_amdgcn_s_getreg((31 << 11) | 4);
    }

    // LDS-DMA source addressing (as conv_gemm_big.hip): piece q of wave w covers rows
    // (w + 8q)*16 .. +15 of the operand; lane l fills physical chunk (l & 3) of row
    // (l >> 2), which holds logical chunk dma_c
    const int dma_row = lane >> 2;
    const int dma_c = ((lane & 3) - 2 * ((lane >> 4) & 3)) & 3;
    int a_src[2];
    int64_t b_off[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        int m = m0 + (wid + 8 * q) * 16 + dma_row;
        m = m < p.M ? m : p.M - 1;  // rows past M read a valid row; never stored
        a_src[q] = src_row(p, m);
        b_off[q] = (int64_t)(n0 + (wid + 8 * q) * 16 + dma_row) * p.Kp + dma_c * 8;
    }
    const CT* A = (const CT*)p.A;
    const CT* W = (const CT*)p.W;
    auto issue_a = [&](int s) {
        const int k0 = s * PK;
        const int tap = k0 / p.Ktap;
        const int cin = k0 - tap * p.Ktap + dma_c * 8;
        char* slot = smem + (s % PSLOTS) * PSLOT_BYTES;
#pragma unroll
        for (int q = 0; q < 2; ++q)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(A + (int64_t)(a_src[q] + tap * p.dil) * p.lda + cin),
                                             (lds_ptr_t)(slot + (wid + 8 * q) * 1024), 16, 0, 0);
    };
    auto issue_b = [&](int s) {
        char* slot = smem + (s % PSLOTS) * PSLOT_BYTES + PM * PK * 2;
#pragma unroll
        for (int q = 0; q < 2; ++q)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(W + b_off[q] + s * PK),
                                             (lds_ptr_t)(slot + (wid + 8 * q) * 1024), 16, 0, 0);
    };

    const int frag_chunk = ((lane >> 4) + 2 * (((lane & 15) >> 2) & 3)) & 3;
    const int a_frag_off = (wr * 128 + (lane & 15)) * 64 + frag_chunk * 16;
    const int b_frag_off = PM * PK * 2 + (wc * 64 + (lane & 15)) * 64 + frag_chunk * 16;

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = p.Kp / PK;
    // prologue: stages 0 and 1 whole, the B pieces of stage 2
    issue_a(0);
    issue_b(0);
    if (nk > 1) {
        issue_a(1);
        issue_b(1);
    }
    if (nk > 2) {
        issue_b(2);
        vmw<6>();
    } else if (nk > 1) {
        vmw<4>();
    } else {
        vmw<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // scale/shift stores
    barrier_pinned();
    if (ABL == 7 && tid == 0) trace_stamp(blockIdx.x, 1);
    if (wr == 1) barrier_pinned();  // G1 runs one barrier interval behind G0

    u32x4 bf[4], alo[4], ahi[4];
    u32x4 res[8][2];
    for (int s = 0; s < nk; ++s) {
        const char* slot = smem + (s % PSLOTS) * PSLOT_BYTES;
        // ---- segment A: B fragments + A rows 0-63 of stage s; A pieces of stage s+2
        if (ABL < 3 || s == 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) bf[j] = *(const u32x4*)(slot + b_frag_off + j * 16 * 64);
#pragma unroll
            for (int i = 0; i < 4; ++i) alo[i] = *(const u32x4*)(slot + a_frag_off + i * 16 * 64);
        }
        if (ABL != 1 && ABL != 4 && s + 2 < nk) issue_a(s + 2);
        // the residual block of this wave, two K-steps before the end (buffer loads,
        // 32-bit offsets: 0 spills); they have the last K-step to land
        if (p.R && s == (nk >= 2 ? nk - 2 : 0)) load_residual_tp_buf<CT, 8>(p, res, m0 + wr * 128, n0 + wc * 64, lane);
        barrier_pinned();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (ABL != 2) acc[i][j] = mfma16<CT>(bf[j], alo[i], acc[i][j]);
                else asm volatile("" ::"v"(bf[j]), "v"(alo[i]));
            }
        __builtin_amdgcn_s_setprio(0);
        barrier_pinned();
        // ---- segment B: A rows 64-127 of stage s; B pieces of stage s+3; wait stage s+1
        if (ABL < 3 || s == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) ahi[i] = *(const u32x4*)(slot + a_frag_off + (4 + i) * 16 * 64);
        }
        if (s + 3 < nk) {
            if (ABL != 1 && ABL != 4) issue_b(s + 3);
            vmw<6>();  // younger than stage s+1: B(s+2), A(s+2), B(s+3)
        } else if (s + 2 < nk) {
            vmw<4>();  // B(s+2), A(s+2)
        } else if (s + 2 == nk) {
            // stage s+1 is the last one; the 16 residual loads issued in segment A of
            // this step are younger and stay in flight (the compiler waits for them
            // before the epilogue reads them)
            if (p.R) vmw<16>();
            else vmw<0>();
        }
        barrier_pinned();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (ABL != 2) acc[4 + i][j] = mfma16<CT>(bf[j], ahi[i], acc[4 + i][j]);
                else asm volatile("" ::"v"(bf[j]), "v"(ahi[i]));
            }
        __builtin_amdgcn_s_setprio(0);
        barrier_pinned();
    }
    if (wr == 0) barrier_pinned();  // match G1's extra barrier
    if (ABL == 7 && tid == 0) trace_stamp(blockIdx.x, 2);

    const __amdgpu_buffer_rsrc_t y_rsrc = make_rsrc(p.Y, (uint32_t)((size_t)p.M * p.ldy * sizeof(CT)));
    epilogue_tp<CT, 8, true, -1, 0>(p, acc, m0 + wr * 128, n0 + wc * 64, lane, s_scale, s_shift, y_rsrc, res);
    if (ABL == 7) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) trace_stamp(blockIdx.x, 3);
    }
}

}  // namespace

// measurement only: where VP3D_ABL=7 launches write their timestamps (10 u64 per workgroup)
hipError_t conv_gemm_8p_set_trace(unsigned long long* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &buf, sizeof(buf));
}

bool conv_gemm_8p_eligible(const ConvGemmParams& p, Act a_type, Act out_type, Act compute) {
    if (compute == Act::F32 || a_type != compute || out_type != compute) return false;
    if (p.Ktap % PK != 0 || p.Kp % PK != 0 || p.lda % 8 != 0) return false;
    if (p.N % PN != 0 || p.N > PMAXN || p.ldy % 8 != 0 || (p.R && p.ldr % 8 != 0)) return false;
    if ((reinterpret_cast<uintptr_t>(p.A) & 15) || (reinterpret_cast<uintptr_t>(p.Y) & 15) ||
        (p.R && (reinterpret_cast<uintptr_t>(p.R) & 15)))
        return false;
    if ((size_t)p.M * p.ldy * 2 >= (1u << 31)) return false;  // 32-bit buffer offsets
    if (p.R && (size_t)((p.M + p.T_out - 1) / p.T_out) * p.R_T * p.ldr * 2 >= (1u << 31)) return false;
    return true;
}

hipError_t launch_conv_gemm_8p(const ConvGemmParams& p, Act compute, hipStream_t stream) {
    const dim3 grid(((p.M + PM - 1) / PM) * (p.N / PN));
#ifdef VP3D_ABLATION
    // measurement builds only (tools/ubench/gemm_check): VP3D_ABL selects an ablated loop
    static const int abl = [] {
        const char* e = getenv("VP3D_ABL");
        return e ? atoi(e) : 0;
    }();
    if (compute == Act::BF16 && abl != 0) {
        switch (abl) {
            case 1: hipLaunchKernelGGL((conv_gemm_8p<__bf16, 1>), grid, dim3(512), 0, stream, p); break;
            case 2: hipLaunchKernelGGL((conv_gemm_8p<__bf16, 2>), grid, dim3(512), 0, stream, p); break;
            case 3: hipLaunchKernelGGL((conv_gemm_8p<__bf16, 3>), grid, dim3(512), 0, stream, p); break;
            case 4: hipLaunchKernelGGL((conv_gemm_8p<__bf16, 4>), grid, dim3(512), 0, stream, p); break;
            default: hipLaunchKernelGGL((conv_gemm_8p<__bf16, 7>), grid, dim3(512), 0, stream, p);
        }
        return hipGetLastError();
    }
#endif
    // (nontemporal output stores, VP3D_GEMM_NT in round 1, measured slower on every layer:
    // b4 k3 0.072 -> 0.083 ms, b1 k3 1.22 -> 1.25-1.29 ms)
    if (compute == Act::BF16)
        hipLaunchKernelGGL((conv_gemm_8p<__bf16>), grid, dim3(512), 0, stream, p);
    else
        hipLaunchKernelGGL((conv_gemm_8p<_Float16>), grid, dim3(512), 0, stream, p);
    return hipGetLastError();
}

}  // namespace vp3d
