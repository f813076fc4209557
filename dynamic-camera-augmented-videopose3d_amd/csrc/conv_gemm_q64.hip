// 256x256 conv-GEMM with 64-deep K-tiles staged as whole 128-byte lines, quadrant phases
// and a wave-group ping-pong (16-bit operands, 16-bit output).
//
// Contract: ConvGemmParams (kernels.h), tap-aligned 16-bit activations (Ktap % 64 == 0):
// the block k-convs and 1x1 convs of TemporalModel / TemporalModelOptimized1f (reference
// common/models/TemporalModel.py:113-119, :129-135, :179-181, :191-195).
//
// Why: conv_gemm_8p stages 32-deep K-steps, so every LDS-DMA instruction fetches 16 rows
// x 64 B — half cache lines — and its K loop measured ~54 % of the MFMA rate (0.94 us per
// 32-deep step at block-1 shapes, tools/ubench/gemm_check trace), limited by the operand
// stream (~42 GB/s per CU), not the MFMAs.  Here a DMA instruction moves 8 rows x 128 B,
// whole lines (cdna_hip_programming.md §5, "x through LDS in full 128-B lines": fragment-
// shaped 16 x 64-B pieces cost +18-45 %, TA_BUSY 2x).
//
// Geometry: 512 threads = 8 waves, wave (wr, wc) = (wid >> 2, wid & 3) owns rows
// 128 wr .. +127 and channels 64 wc .. +63; MFMA v_mfma_f32_16x16x32 issued transposed
// (D = W . A^T) so the epilogue is gemm::epilogue_tp (registers only).
// LDS: 2 buffers x (A 256 rows + W 256 rows) x 128 B = 128 KiB; 16-byte chunk c of row r
// stored at chunk c ^ ((r >> 1) & 7) (conflict-free ds_read_b128 for the fragment reads;
// the swizzle is applied to each lane's SOURCE address, the DMA writes lane-linearly).
//
// K-tile t = 3 phases over the quadrants of the wave's 128 x 64 tile (rows h, channels g):
//   Q0  (h0, g0):            read A_h0 (8 ds_read_b128) + W_g0 (4)   issue A_h0 of tile t+1
//   Q1  (h0, g1):            read W_g1 (4)                            issue W_g0 of t+1
//   Q23 (h1, g1) + (h1, g0): read A_h1 (8)                            issue W_g1, A_h1 of t+1
// W_g0 stays in 16 more VGPRs from Q0 to Q23 (re-reading it measured 0.6-0.9 % slower), and
// Q2 / Q3 share one 32-MFMA phase (two barriers fewer per K-tile: block-1 k3 -3.3 %).  A
// region (A_h* / W_g*) is re-staged >= 2 phases after its last read, its reads retired
// before the barrier that ends their phase (WAR), and read >= 2 phases after its DMA was
// issued; each wave waits (vmcnt(4), never 0 in steady state) in the memory segment of the
// phase BEFORE the one that reads the region, which precedes that read by a barrier for both
// wave groups (RAW).  Each phase: [reads + DMA pieces + wait] barrier lgkmcnt(0) [16 or 32
// MFMAs at s_setprio 1] barrier; wave group 1 runs one barrier
// behind group 0, so the two waves of a SIMD alternate memory and MFMA segments.
#include <cstdlib>
#include <cstring>

#include "gemm_common.h"

namespace vp3d {
namespace {

using namespace gemm;

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int QM = 256, QN = 256, QK = 64;
constexpr int QBUF = (QM + QN) * QK * 2;  // 64 KiB per buffer
constexpr int QW_OFF = QM * QK * 2;       // W region inside a buffer
constexpr int QMAXN = 1024;

__device__ __forceinline__ void qbarrier() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void qvm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// EPI (measurement builds only, tools/ubench/gemm_check with VP3D_ABL): 0 = the epilogue,
// 1 = stores issued but dropped by the range check (no output traffic), 2 = no epilogue,
// 3 = the epilogue without the residual loads
#ifdef VP3D_ABLATION
// measurement builds only: first-round workgroups of CU group g = (bid >> 3) % groups sleep
// g * iters x 127 x 64 cycles before starting, so their tiles' epilogues (output + residual
// traffic) fall at different times across the chip (VP3D_STAGGER=iters[,groups])
__device__ int g_stagger_iters;
__device__ int g_stagger_groups;
#endif

// X3 (split fp16, VP3D_DTYPE_F16X3): A and W rows hold every f32 value x as two f16
// halves hi = f16(x), lo = f16(x - hi), each 32-wide K group stored [hi(32) | lo(32)] --
// exactly a 16-bit operand of twice the K -- so the DMA, LDS layout and fragment reads
// are the plain kernel's, with kh = 0 the hi and kh = 1 the lo fragments of 32 K values.
// The MFMA pattern per fragment pair is hi.hi + hi.lo + lo.hi (the lo.lo term, 2^-22
// relative, is dropped): 3 MFMAs per 2 fragment reads instead of 2.
// X3 = 1: split output rows; X3 = 2: f32 output rows (the layer before the shrink).
template <typename CT, int EPI = 0, int X3 = 0>
__global__ __launch_bounds__(512, 1) void conv_gemm_q64(ConvGemmParams p) {
#ifdef VP3D_ABLATION
    if (g_stagger_iters > 0 && blockIdx.x < 256) {
        const int n = ((blockIdx.x >> 3) % g_stagger_groups) * g_stagger_iters;
        for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(127);
    }
#endif
    __shared__ __attribute__((aligned(16))) char smem[2 * QBUF + 2 * QMAXN * 4];
    float* const s_scale = (float*)(smem + 2 * QBUF);
    float* const s_shift = s_scale + QMAXN;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wr = wid >> 2, wc = wid & 3;

    for (int i = tid; i < p.N; i += 512) {
        s_scale[i] = p.scale[i];
        s_shift[i] = p.shift[i];
    }

    const int ntn = (p.N + QN - 1) / QN;  // X3: N % 64 == 0, waves past N skip the epilogue
    const int ntm = (p.M + QM - 1) / QM;
    const int wg = xcd_remap(blockIdx.x, ntm * ntn);
    const int tile_m = wg / ntn;
    const int tile_n = wg - tile_m * ntn;
    const int m0 = tile_m * QM, n0 = tile_n * QN;

    // ---- DMA pieces: 8 rows x 128 B each.  Region pieces (of 32 per operand):
    //   A_h0 = {0..7, 16..23}, A_h1 = {8..15, 24..31}   (rows 64-row halves of each wave row)
    //   W_g0 = {8c + 0..3},     W_g1 = {8c + 4..7}       (channel halves of each wave column)
    // wave w issues two pieces of each region: A_h0 {w, 16+w}, A_h1 {8+w, 24+w},
    // W_g0 {8(w>>2)+(w&3), 16+8(w>>2)+(w&3)}, W_g1 the same + 4.
    // Lane l fills row 8q + (l >> 3), physical chunk (l & 7) = logical chunk lc ^ swz.
    const int prow = lane >> 3;
    auto lchunk = [&](int q) { return (lane & 7) ^ (((q & 1) * 4 + (prow >> 1)) & 7); };
    int a_q[4];
    a_q[0] = wid; a_q[1] = 16 + wid;          // A_h0
    a_q[2] = 8 + wid; a_q[3] = 24 + wid;      // A_h1
    int w_q[4];
    w_q[0] = 8 * (wid >> 2) + (wid & 3); w_q[1] = w_q[0] + 16;  // W_g0
    w_q[2] = w_q[0] + 4; w_q[3] = w_q[1] + 4;                  // W_g1
    // every piece of a wave has the parity of wid (A) / of wid & 3 (W): one chunk each
    const int a_lc = lchunk(wid), w_lc = lchunk(wid & 3);
    int a_src[4], w_off[4];  // W extent Np * Kp < 2^31 elements
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int m = m0 + 8 * a_q[j] + prow;
        m = m < p.M ? m : p.M - 1;  // rows past M read a valid row; never stored
        a_src[j] = src_row(p, m);
        w_off[j] = (n0 + 8 * w_q[j] + prow) * p.Kp + w_lc * 8;  // W rows padded to 256
    }
    const CT* A = (const CT*)p.A;
    const CT* W = (const CT*)p.W;
    // region r of tile s: 0 = A_h0, 1 = W_g0, 2 = W_g1, 3 = A_h1 (issue order)
    auto issue = [&](int s, int r) {
        char* buf = smem + (s & 1) * QBUF;
        const int k0 = s * QK;
        if (r == 0 || r == 3) {
            const int j0 = r == 0 ? 0 : 2;
            const int tap = k0 / p.Ktap;
            const int cb = k0 - tap * p.Ktap;
#pragma unroll
            for (int j = j0; j < j0 + 2; ++j)
                __builtin_amdgcn_global_load_lds(
                    (gbl_ptr_t)(A + (int64_t)(a_src[j] + tap * p.dil) * p.lda + cb + a_lc * 8),
                    (lds_ptr_t)(buf + a_q[j] * 1024), 16, 0, 0);
        } else {
            const int j0 = r == 1 ? 0 : 2;
#pragma unroll
            for (int j = j0; j < j0 + 2; ++j)
                __builtin_amdgcn_global_load_lds((gbl_ptr_t)(W + w_off[j] + k0),
                                                 (lds_ptr_t)(buf + QW_OFF + w_q[j] * 1024), 16, 0, 0);
        }
    };

    // ---- fragment reads: row (l & 15) of a 16-row block, logical chunk 4 kh + (l >> 4),
    // physical chunk ^ ((l & 15) >> 1) (row blocks start at multiples of 16) ----
    const int fsw = (lane & 15) >> 1;
    const int fo0 = (lane & 15) * 128 + (((lane >> 4) ^ fsw) << 4);        // kh = 0
    const int fo1 = (lane & 15) * 128 + ((((lane >> 4) + 4) ^ fsw) << 4);  // kh = 1
    const int a_base = wr * 128 * 128;
    const int w_base = QW_OFF + wc * 64 * 128;

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    u32x4 af[4][2];  // A fragments of the current row half: [row block][kh]
    u32x4 bf[2][2][2];  // W fragments of both channel halves: [g][block jj][kh]

    auto read_a = [&](const char* buf, int h) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const char* r = buf + a_base + (h * 64 + i * 16) * 128;
            af[i][0] = *(const u32x4*)(r + fo0);
            af[i][1] = *(const u32x4*)(r + fo1);
        }
    };
    // both channel halves' W fragments stay in registers for the whole K-tile, so the h1
    // quadrants read only A_h1 (24 instead of 28 KiB of LDS reads per wave per K-tile;
    // re-reading W_g0 instead of holding 16 more VGPRs measured 0.6-0.9 % slower)
    auto read_w = [&](const char* buf, int g) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
            const char* r = buf + w_base + (g * 32 + jj * 16) * 128;
            bf[g][jj][0] = *(const u32x4*)(r + fo0);
            bf[g][jj][1] = *(const u32x4*)(r + fo1);
        }
    };
    auto mma = [&](int h, int g) {
        __builtin_amdgcn_s_setprio(1);
        if constexpr (X3 != 0) {
            // term t: (W, A) halves (hi, hi), (hi, lo), (lo, hi); 8 independent
            // accumulators between two MFMAs on the same one
#pragma unroll
            for (int t = 0; t < 3; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj)
                        acc[4 * h + i][2 * g + jj] = mfma16<CT>(bf[g][jj][t == 2 ? 1 : 0], af[i][t == 1 ? 1 : 0],
                                                                acc[4 * h + i][2 * g + jj]);
        } else {
#pragma unroll
            for (int kh = 0; kh < 2; ++kh)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj)
                        acc[4 * h + i][2 * g + jj] =
                            mfma16<CT>(bf[g][jj][kh], af[i][kh], acc[4 * h + i][2 * g + jj]);
        }
        __builtin_amdgcn_s_setprio(0);
    };
    auto compute_seg = [&](int h, int g) {
        qbarrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        mma(h, g);
        qbarrier();
    };

    const int nk = p.Kp / QK;
    // prologue: tile 0 whole (A_h0, W_g0, W_g1, A_h1); A_h0 and W_g0 landed
    issue(0, 0);
    issue(0, 1);
    issue(0, 2);
    issue(0, 3);
    qvm<4>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // scale / shift stores
    qbarrier();
    if (wr == 1) qbarrier();  // group 1 runs one barrier behind group 0

    for (int t = 0; t < nk; ++t) {
        const char* buf = smem + (t & 1) * QBUF;
        const bool more = t + 1 < nk;
        // ---- Q0: A_h0 + W_g0; stage A_h0(t+1); wait W_g1(t) ----
        read_a(buf, 0);
        read_w(buf, 0);
        if (more) {
            issue(t + 1, 0);
            qvm<4>();  // W_g1(t) landed: younger A_h1(t), A_h0(t+1)
        } else {
            qvm<2>();  // younger: A_h1(t)
        }
        compute_seg(0, 0);
        // ---- Q1: W_g1; stage W_g0(t+1); wait A_h1(t) ----
        read_w(buf, 1);
        if (more) {
            issue(t + 1, 1);
            qvm<4>();  // younger: A_h0(t+1), W_g0(t+1)
        } else {
            qvm<0>();
        }
        compute_seg(0, 1);
        // ---- Q2 + Q3 as one phase of 32 MFMAs (h1 x both channel halves; W_g0 still in
        // registers since Q0): A_h1; stage W_g1(t+1), A_h1(t+1); wait A_h0(t+1), W_g0(t+1) ----
        read_a(buf, 1);
        if (more) {
            issue(t + 1, 2);
            issue(t + 1, 3);
            qvm<4>();  // younger: W_g1(t+1), A_h1(t+1)
        }
        qbarrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        mma(1, 1);
        mma(1, 0);
        qbarrier();
    }
    if (wr == 0) qbarrier();  // match group 1's extra barrier

    if constexpr (X3 != 0) {
        if (n0 + wc * 64 >= p.N) return;  // a wave's 64 channels lie wholly past N
        constexpr int OB = X3 == 2 ? 4 : 2;  // output element bytes
        const size_t y_rest = (size_t)(p.M - m0) * p.ldy * OB;
        const __amdgpu_buffer_rsrc_t y_rsrc =
            make_rsrc((const char*)p.Y + (size_t)m0 * p.ldy * OB,
                      (uint32_t)(y_rest < 0x7FFFFFFFu ? y_rest : 0x7FFFFFFFu));
        if (p.R)
            epilogue_tp_x3<X3 == 2, 1>(p, acc, m0 + wr * 128, n0 + wc * 64, lane, s_scale, s_shift, y_rsrc, m0);
        else
            epilogue_tp_x3<X3 == 2, 0>(p, acc, m0 + wr * 128, n0 + wc * 64, lane, s_scale, s_shift, y_rsrc, m0);
        return;
    }
    // the output resource starts at the tile's first row (outputs past 2^31 bytes: the
    // store offsets stay 32-bit and tile-relative; rows past M fall outside the range)
    const size_t y_rest = (size_t)(p.M - m0) * p.ldy * sizeof(CT);
    const __amdgpu_buffer_rsrc_t y_rsrc =
        make_rsrc((const CT*)p.Y + (size_t)m0 * p.ldy,
                  EPI == 1 ? 0u : (uint32_t)(y_rest < 0x7FFFFFFFu ? y_rest : 0x7FFFFFFFu));
    if (EPI == 2) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
        return;
    }
    // the residual (1x1 convs) is loaded inside the epilogue, one row block ahead of its
    // use (issuing all 16 loads of the block when the K loop ends measured the same:
    // block-1 1x1 + residual 0.674 vs 0.667 ms -- per-CU bandwidth, not latency)
    if (p.R && EPI != 3)
        epilogue_tp<CT, 8, false, 1, 0>(p, acc, m0 + wr * 128, n0 + wc * 64, lane, s_scale, s_shift, y_rsrc,
                                        nullptr, m0);
    else
        epilogue_tp<CT, 8, false, 0, 0>(p, acc, m0 + wr * 128, n0 + wc * 64, lane, s_scale, s_shift, y_rsrc,
                                        nullptr, m0);
}

}  // namespace

bool conv_gemm_q64_eligible(const ConvGemmParams& p, Act a_type, Act out_type, Act compute) {
    if (compute == Act::F32 || a_type != compute || out_type != compute) return false;
    if (p.Ktap % QK != 0 || p.Kp % QK != 0 || p.lda % 8 != 0) return false;
    if (p.N % QN != 0 || p.N > QMAXN || p.ldy % 8 != 0 || (p.R && p.ldr % 8 != 0)) return false;
    if ((reinterpret_cast<uintptr_t>(p.A) & 15) || (reinterpret_cast<uintptr_t>(p.Y) & 15) ||
        (p.R && (reinterpret_cast<uintptr_t>(p.R) & 15)))
        return false;
    // any output size: the store resource is rebased per tile, A / W / residual
    // addresses are 64-bit (A rows and Np * Kp stay below 2^31)
    return (size_t)p.N * p.Kp < (1u << 31);
}

bool conv_gemm_q64_x3_eligible(const ConvGemmParams& p, bool out_f32) {
    if (p.Ktap % QK != 0 || p.Kp % QK != 0 || p.lda % 8 != 0) return false;
    if (p.N % 64 != 0 || p.N > QMAXN || p.ldy % (out_f32 ? 4 : 8) != 0 || (p.R && p.ldr % 8 != 0)) return false;
    if ((reinterpret_cast<uintptr_t>(p.A) & 15) || (reinterpret_cast<uintptr_t>(p.Y) & 15) ||
        (reinterpret_cast<uintptr_t>(p.W) & 15) || (p.R && (reinterpret_cast<uintptr_t>(p.R) & 15)))
        return false;
    return (size_t)((p.N + QN - 1) / QN * QN) * p.Kp < (1u << 31);
}

hipError_t launch_conv_gemm_q64_x3(const ConvGemmParams& p, bool out_f32, hipStream_t stream) {
    const dim3 grid(((p.M + QM - 1) / QM) * ((p.N + QN - 1) / QN));
    if (out_f32)
        hipLaunchKernelGGL((conv_gemm_q64<_Float16, 0, 2>), grid, dim3(512), 0, stream, p);
    else
        hipLaunchKernelGGL((conv_gemm_q64<_Float16, 0, 1>), grid, dim3(512), 0, stream, p);
    return hipGetLastError();
}

hipError_t launch_conv_gemm_q64(const ConvGemmParams& p, Act compute, hipStream_t stream) {
    const dim3 grid(((p.M + QM - 1) / QM) * (p.N / QN));
#ifdef VP3D_ABLATION
    static const int abl = [] {
        const char* e = getenv("VP3D_ABL");
        const char* st = getenv("VP3D_STAGGER");
        if (st) {
            int it = atoi(st), gr = 2;
            if (const char* c = strchr(st, ',')) gr = atoi(c + 1);
            if (gr < 1) gr = 1;
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stagger_iters), &it, sizeof(int));
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stagger_groups), &gr, sizeof(int));
        }
        return e ? atoi(e) : 0;
    }();
    if (compute == Act::BF16 && (abl >= 1 && abl <= 3)) {
        if (abl == 1) hipLaunchKernelGGL((conv_gemm_q64<__bf16, 1>), grid, dim3(512), 0, stream, p);
        else if (abl == 2) hipLaunchKernelGGL((conv_gemm_q64<__bf16, 2>), grid, dim3(512), 0, stream, p);
        else hipLaunchKernelGGL((conv_gemm_q64<__bf16, 3>), grid, dim3(512), 0, stream, p);
        return hipGetLastError();
    }
#endif
    if (compute == Act::BF16)
        hipLaunchKernelGGL((conv_gemm_q64<__bf16>), grid, dim3(512), 0, stream, p);
    else
        hipLaunchKernelGGL((conv_gemm_q64<_Float16>), grid, dim3(512), 0, stream, p);
    return hipGetLastError();
}

}  // namespace vp3d
