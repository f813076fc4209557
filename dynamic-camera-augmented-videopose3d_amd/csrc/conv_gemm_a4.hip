// 256x256 conv-GEMM at ONE wave per SIMD with the accumulators in named AGPRs
// (16-bit operands, 16-bit output).
//
// Contract: that of conv_gemm_q64 (ConvGemmParams, kernels.h): tap-aligned 16-bit
// activations (Ktap % 64 == 0), N % 256 == 0 -- the block k-convs and 1x1 convs of
// TemporalModel / TemporalModelOptimized1f (reference common/models/TemporalModel.py:113-119,
// :129-135, :179-181, :191-195).
//
// Why: q64 keeps two waves per SIMD alternating memory and MFMA segments, six barriers per
// 64-deep K-tile; its K loop leaves the matrix cores idle ~42 % of the cycles, and its MFMA +
// barrier skeleton alone (no memory traffic) already ran at ~0.7 of the MFMA rate.  Here 4
// waves each own a 128 x 128 output tile (the shape of hipBLASLt's MT256x256x64 kernels),
// with ONE barrier per K-tile: the single wave on a SIMD keeps the MFMA pipe fed by itself,
// its next fragment set and the LDS-DMA of the K-tile after next issued between its MFMAs.
// A 128 x 128 wave tile also reads a third fewer LDS bytes per MFMA than q64's 128 x 64.
//
// Registers: the 256 accumulators per lane (8 row blocks x 8 channel blocks x 4) live in
// AGPRs a0..a255 named in the MFMA text (block (i, j) at a[4 (8 i + j) .. +3]); the compiler
// never sees them (they are clobbered once at entry so the kernel descriptor allocates
// them), which is what the retired compiler-allocated form lacked (tools/ubench/retired/
// conv_gemm_q4w.hip: 201 VGPR spills, 4.4x slower).  Fragments: two sets of 8 A + 8 W
// u32x4 (128 VGPRs), read by plain LDS loads the compiler counts and waits for.
//
// K-tile t (64 deep, LDS buffer t & 1, staged by LDS-DMA as whole 128-byte lines with
// q64's chunk swizzle):
//   phase A: 64 MFMAs on set 0 (k 0..31 of t), reads of set 1 (k 32..63 of t)
//   mid:     vmcnt(0) (tile t + 1 landed: this wave's pieces), lgkmcnt(0) (tile t read out
//            by this wave), barrier
//   phase B: 64 MFMAs on set 1, reads of set 0 (k 0..31 of t + 1) and this wave's 16 DMA
//            pieces of tile t + 2 into buffer t & 1, which every wave has finished reading
// (reads and DMA pieces one per two MFMAs).  Measured (MI355X, random bf16, block-1 shapes at
// B = 8192, tools/ubench/gemm_check): k3 1.18 ms vs q64 1.29 ms, 1x1 + residual 0.62-0.63 vs
// 0.66-0.69; MFMA pipes busy 0.68 of the cycles vs 0.57, at a lower clock (1.68 vs 1.81 GHz:
// the chip holds its power); ablations: without the loop DMA 1.00 ms, without the fragment
// reads 1.11, without both 0.90.
// Epilogue: the accumulators copied to VGPRs 128 at a time, gemm::epilogue_tp per 64
// channels (BN/ReLU, residual, 16-byte stores), as q64.
#include <cstdlib>
#include <cstring>
#include <utility>

#include "gemm_common.h"

namespace vp3d {
namespace {

using namespace gemm;

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int GM = 256, GN = 256, GK = 64;
constexpr int GBUF = (GM + GN) * GK * 2;  // 64 KiB per buffer
constexpr int GW_OFF = GM * GK * 2;       // W region inside a buffer
constexpr int GMAXN = 1024;
// s_waitcnt immediates (gfx9 encoding: vmcnt [3:0] + [15:14], expcnt [6:4], lgkmcnt [11:8])
constexpr int kLgkm0 = 0xC07F;     // lgkmcnt(0)
constexpr int kVm0Lgkm0 = 0x0070;  // vmcnt(0) lgkmcnt(0)
constexpr int kVm16Lgkm0 = 0x4070; // vmcnt(16) lgkmcnt(0)

template <typename F, int... Is>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ void pinned_barrier() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

// a[R..R+3] (+)= W . A^T; ZERO: C = 0 (the first K-tile initialises every block)
template <typename CT, int R, bool ZERO>
__device__ __forceinline__ void amma(const u32x4& w, const u32x4& a) {
    if constexpr (std::is_same<CT, __bf16>::value) {
        if constexpr (ZERO)
            asm volatile("v_mfma_f32_16x16x32_bf16 a[%c2:%c3], %0, %1, 0" ::"v"(w), "v"(a), "i"(R), "i"(R + 3));
        else
            asm volatile("v_mfma_f32_16x16x32_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(w), "v"(a), "i"(R),
                         "i"(R + 3));
    } else {
        if constexpr (ZERO)
            asm volatile("v_mfma_f32_16x16x32_f16 a[%c2:%c3], %0, %1, 0" ::"v"(w), "v"(a), "i"(R), "i"(R + 3));
        else
            asm volatile("v_mfma_f32_16x16x32_f16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(w), "v"(a), "i"(R),
                         "i"(R + 3));
    }
}

template <int R>
__device__ __forceinline__ float aread() {
    float x;
    asm volatile("v_accvgpr_read_b32 %0, a%c1" : "=v"(x) : "i"(R));
    return x;
}

// clobber names a0 .. a255 (A4_C10(d) = a<d>0 .. a<d>9)
#define A4_C10(d) "a" #d "0", "a" #d "1", "a" #d "2", "a" #d "3", "a" #d "4", "a" #d "5", "a" #d "6", "a" #d "7", \
                  "a" #d "8", "a" #d "9"
#define A4_ALL_AGPRS                                                                                              \
    "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", A4_C10(1), A4_C10(2), A4_C10(3), A4_C10(4),      \
        A4_C10(5), A4_C10(6), A4_C10(7), A4_C10(8), A4_C10(9), A4_C10(10), A4_C10(11), A4_C10(12), A4_C10(13),   \
        A4_C10(14), A4_C10(15), A4_C10(16), A4_C10(17), A4_C10(18), A4_C10(19), A4_C10(20), A4_C10(21),          \
        A4_C10(22), A4_C10(23), A4_C10(24), "a250", "a251", "a252", "a253", "a254", "a255"

#ifdef VP3D_ABLATION
// measurement builds: ABL bit 2 = per-workgroup stamps into g_a4_trace (10 u64 each:
// 0-3 wall clock (100 MHz) at start / prologue done / K loop done / stores retired, 4 hardware
// ids, 5-8 shader-clock cycles at the same points, 9 cycles wave 0 spent in the mid waits +
// barriers; tools/ubench/gemm_check a4t)
__device__ unsigned long long* g_a4_trace;
#endif

template <typename CT, int ABL>
__global__ __launch_bounds__(256, 1) void conv_gemm_a4(ConvGemmParams p) {
    // the accumulator file is this kernel's own from here on (see the header)
    asm volatile("" ::: A4_ALL_AGPRS);

    __shared__ __attribute__((aligned(16))) char smem[2 * GBUF + 2 * GMAXN * 4];
    float* const s_scale = (float*)(smem + 2 * GBUF);
    float* const s_shift = s_scale + GMAXN;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wr = wid >> 1, wc = wid & 1;
    const int widu = __builtin_amdgcn_readfirstlane(wid);  // wave-uniform: LDS-DMA destinations in SGPRs

    for (int i = tid; i < p.N; i += 256) {
        s_scale[i] = p.scale[i];
        s_shift[i] = p.shift[i];
    }

    const int ntn = p.N / GN;
    const int ntm = (p.M + GM - 1) / GM;
    const int wg = xcd_remap(blockIdx.x, ntm * ntn);
    const int tile_m = wg / ntn;
    const int tile_n = wg - tile_m * ntn;
    const int m0 = tile_m * GM, n0 = tile_n * GN;
#ifdef VP3D_ABLATION
    unsigned long long* const trc = (ABL & 4) && g_a4_trace ? g_a4_trace + (size_t)blockIdx.x * 10 : nullptr;
    unsigned long long mid_cyc = 0;
    auto stamp = [&](int slot) __attribute__((always_inline)) {
        if (trc && tid == 0) {
            trc[slot] = __builtin_amdgcn_s_memrealtime();
            trc[slot + 5] = __builtin_amdgcn_s_memtime();
        }
    };
    stamp(0);
    if (trc && tid == 0)
        trc[4] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                 __builtin_amdgcn_s_getreg((31 << 11) | 4);
#endif

    // ---- DMA pieces: 8 rows x 128 B each, 32 per operand; wave w issues q = w + 4 i.
    // Lane l fills row 8q + (l >> 3), physical chunk (l & 7) = logical chunk lc ^ swz; all
    // pieces of a wave share the parity of q (= that of w): one swizzled chunk each ----
    const int prow = lane >> 3;
    const int lc = (lane & 7) ^ (((wid & 1) * 4 + (prow >> 1)) & 7);
    // LDS-DMA as buffer_load ... lds through per-tile resources: 32-bit lane offsets fixed
    // for the launch, the tile's k offset in soffset, so no per-piece address arithmetic
    // (global_load_lds from 64-bit lane pointers measured 2 % slower: block-1 k3 shape,
    // B = 8192, 1.251-1.262 vs 1.231-1.237 ms)
    uint32_t va[8], vw[8];
    const int srow0 = src_row(p, m0);  // m0 < M; wave-uniform
    const __amdgpu_buffer_rsrc_t a_rsrc = make_rsrc((const CT*)p.A + (int64_t)srow0 * p.lda, 0x7FFFFFFFu);
    const __amdgpu_buffer_rsrc_t w_rsrc = make_rsrc((const CT*)p.W + (int64_t)n0 * p.Kp, 0x7FFFFFFFu);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        int m = m0 + 8 * (wid + 4 * i) + prow;
        m = m < p.M ? m : p.M - 1;  // rows past M read a valid row; never stored
        va[i] = (uint32_t)(((src_row(p, m) - srow0) * p.lda + lc * 8) * (int)sizeof(CT));
        vw[i] = (uint32_t)(((8 * (wid + 4 * i) + prow) * p.Kp + lc * 8) * (int)sizeof(CT));  // W rows padded to 256
    }
    // 1x1 convs (residual): the tile's residual rows land in LDS by LDS-DMA during the last
    // two K-tiles, into the operand buffers those no longer need -- part h (the channel half
    // h of both wave columns: 256 rows x 2 x 128 B = 64 KiB) in phase B of tile nk - 2 + h,
    // in the DMA slots; rows at 128-byte pitch with the operands' chunk swizzle -- so the
    // epilogue reads them from LDS instead of waiting on global loads row block by row block
    const int nk = p.Kp / GK;  // >= 1
    const bool lres = p.R != nullptr && nk >= 3;
    uint32_t vr[8];
    const int rrow0 = lres ? res_row(p, m0) : 0;
    const __amdgpu_buffer_rsrc_t r_rsrc =
        make_rsrc(lres ? (const CT*)p.R + (int64_t)rrow0 * p.ldr : (const CT*)p.A, 0x7FFFFFFFu);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        int m = m0 + 8 * (wid + 4 * i) + prow;
        m = m < p.M ? m : p.M - 1;
        vr[i] = lres ? (uint32_t)(((res_row(p, m) - rrow0) * p.ldr + lc * 8) * (int)sizeof(CT)) : 0u;
    }
    // piece k of part h: wave column k >> 3, the rows of A piece k & 7
    auto res_piece = [&](char* buf, int k, int h) __attribute__((always_inline)) {
        const int wcp = k >> 3;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r_rsrc, (lds_ptr_t)(buf + (wcp * 32 + widu + 4 * (k & 7)) * 1024), 16,
                                                 vr[k & 7], (uint32_t)((n0 + 128 * wcp + 64 * h) * (int)sizeof(CT)),
                                                 0, 0);
    };
    // k offset of tile s inside a row: tap * dil rows + channel base (wave-uniform)
    auto a_koff = [&](int s) __attribute__((always_inline)) -> int64_t {
        const int k0 = s * GK;
        const int tap = k0 / p.Ktap;
        return (int64_t)tap * p.dil * p.lda + (k0 - tap * p.Ktap);
    };
    auto dma_piece = [&](char* buf, int i, int s, int64_t aoff) __attribute__((always_inline)) {
        if (i < 8)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, (lds_ptr_t)(buf + (widu + 4 * i) * 1024), 16, va[i],
                                                     (uint32_t)aoff * (uint32_t)sizeof(CT), 0, 0);
        else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(w_rsrc, (lds_ptr_t)(buf + GW_OFF + (widu + 4 * (i - 8)) * 1024),
                                                     16, vw[i - 8], (uint32_t)(s * GK * (int)sizeof(CT)), 0, 0);
    };

    // ---- fragment reads (q64's layout): row (l & 15) of a 16-row block, logical chunk
    // 4 kh + (l >> 4), physical chunk ^ ((l & 15) >> 1) ----
    const int fsw = (lane & 15) >> 1;
    const int fo0 = (lane & 15) * 128 + (((lane >> 4) ^ fsw) << 4);
    const int fo1 = (lane & 15) * 128 + ((((lane >> 4) + 4) ^ fsw) << 4);
    const int a_base = wr * 128 * 128;
    const int w_base = GW_OFF + wc * 128 * 128;

    u32x4 fa[2][8], fw[2][8];  // [set][block]

    // 64 MFMAs on set CUR; RD: the 16 reads of set NXT from `rbuf` at k-half offset `fo`;
    // DMA: the 16 pieces of tile `s` into `dbuf`, two per row block
    auto phase = [&](auto cur_c, auto zero_c, auto rd_c, auto dma_c, const char* rbuf, int fo, char* dbuf, int s,
                     int resp) __attribute__((always_inline)) {
        constexpr int CUR = decltype(cur_c)::value;
        constexpr int NXT = CUR ^ 1;
        constexpr bool ZERO = decltype(zero_c)::value;
        constexpr bool RD = decltype(rd_c)::value;
        constexpr bool DMA = decltype(dma_c)::value;
        const int64_t aoff = DMA ? a_koff(s) : 0;
        // each row block: the MFMA on channel block j, with one memory instruction ahead of
        // the even ones: A read, DMA piece, W read, DMA piece (bursts of 2 reads + 2 pieces
        // at the row block's start measured 3 % slower at B = 8192, the same at 65,536;
        // 4 pieces in each of the first 4 row blocks 3-6 % slower).  ABL (measurement
        // builds): bit 0 no loop DMA, bit 1 no loop fragment reads
        constexpr bool DO_RD = RD && !(ABL & 2);
        constexpr bool DO_DMA = DMA && !(ABL & 1);
        static_for<8>([&](auto i_c) __attribute__((always_inline)) {
            constexpr int I = decltype(i_c)::value;
            static_for<8>([&](auto j_c) __attribute__((always_inline)) {
                constexpr int J = decltype(j_c)::value;
                if constexpr (DO_RD && J == 0) fa[NXT][I] = *(const u32x4*)(rbuf + a_base + I * 2048 + fo);
                if constexpr (DO_RD && J == 4) fw[NXT][I] = *(const u32x4*)(rbuf + w_base + I * 2048 + fo);
                if constexpr (DO_DMA && (J == 2 || J == 6)) dma_piece(dbuf, 2 * I + J / 4, s, aoff);
                if constexpr (!DMA && (J == 2 || J == 6)) {
                    if (resp >= 0) res_piece(dbuf, 2 * I + J / 4, resp);
                }
                amma<CT, 4 * (8 * I + J), ZERO>(fw[CUR][J], fa[CUR][I]);
                __builtin_amdgcn_sched_barrier(0);
            });
        });
        // the NXT reads (the last issued 8 MFMAs ago) have landed; as a builtin the compiler's
        // own wait bookkeeping sees it, so it adds no lgkmcnt wait behind the next phase's
        // first reads (an asm wait here left it waiting for those at the next phase's
        // first MFMA)
        if constexpr (RD) __builtin_amdgcn_s_waitcnt(kLgkm0);
    };

    char* const buf0 = smem;
    char* const buf1 = smem + GBUF;
    {
        const int64_t o0 = a_koff(0);
#pragma unroll
        for (int i = 0; i < 16; ++i) dma_piece(buf0, i, 0, o0);
    }
    if (nk > 1) {
        const int64_t o1 = a_koff(1);
#pragma unroll
        for (int i = 0; i < 16; ++i) dma_piece(buf1, i, 1, o1);
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 0 landed (younger: tile 1)
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // scale / shift stores
    pinned_barrier();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        fa[0][i] = *(const u32x4*)(buf0 + a_base + i * 2048 + fo0);
        fw[0][i] = *(const u32x4*)(buf0 + w_base + i * 2048 + fo0);
    }

    // last: the 16 residual pieces of part 0 (issued in the phase before) may stay in flight
    auto mid = [&](bool last) __attribute__((always_inline)) {
#ifdef VP3D_ABLATION
        const unsigned long long c0 = (ABL & 4) ? __builtin_amdgcn_s_memtime() : 0;
#endif
        if (last)
            __builtin_amdgcn_s_waitcnt(kVm16Lgkm0);
        else
            __builtin_amdgcn_s_waitcnt(kVm0Lgkm0);
        pinned_barrier();
#ifdef VP3D_ABLATION
        if (ABL & 4) mid_cyc += __builtin_amdgcn_s_memtime() - c0;
#endif
    };
    using C0 = std::integral_constant<int, 0>;
    using C1 = std::integral_constant<int, 1>;
    using T_ = std::integral_constant<bool, true>;
    using F_ = std::integral_constant<bool, false>;
    // K-tile t in buffer `b` (the other one `o`); RD / DMA: tile t + 1 / t + 2 exists;
    // resp >= 0: residual part resp into `b` in phase B
    auto ktile = [&](auto zero_c, auto rd_c, auto dma_c, int t, char* b, char* o, int resp) __attribute__((always_inline)) {
        phase(C0{}, zero_c, T_{}, F_{}, b, fo1, nullptr, 0, -1);
        mid(resp == 1);
        phase(C1{}, F_{}, rd_c, dma_c, o, fo0, b, t + 2, resp);
    };
    const int res0 = lres ? 0 : -1, res1 = lres ? 1 : -1;
#ifdef VP3D_ABLATION
    stamp(1);
#endif
    // tile 0 (phase A initialises the accumulators: C = 0), then the steady state (both
    // follow-up tiles exist: no branch inside a tile), then the last two tiles (with nk >= 3
    // always the tail's last two calls)
    if (nk > 2)
        ktile(T_{}, T_{}, T_{}, 0, buf0, buf1, -1);
    else if (nk == 2)
        ktile(T_{}, T_{}, F_{}, 0, buf0, buf1, -1);
    else
        ktile(T_{}, F_{}, F_{}, 0, buf0, buf1, -1);
    int t = 1;
    for (; t + 3 < nk; t += 2) {
        ktile(F_{}, T_{}, T_{}, t, buf1, buf0, -1);
        ktile(F_{}, T_{}, T_{}, t + 1, buf0, buf1, -1);
    }
    // 0..3 tiles left, t odd (buffer 1)
    if (t + 2 < nk) {  // three: t, t + 1, t + 2
        ktile(F_{}, T_{}, T_{}, t, buf1, buf0, -1);
        ktile(F_{}, T_{}, F_{}, t + 1, buf0, buf1, res0);
        ktile(F_{}, F_{}, F_{}, t + 2, buf1, buf0, res1);
    } else if (t + 1 < nk) {  // two
        ktile(F_{}, T_{}, F_{}, t, buf1, buf0, res0);
        ktile(F_{}, F_{}, F_{}, t + 1, buf0, buf1, res1);
    } else if (t < nk) {  // one (nk <= 2: no residual parts)
        ktile(F_{}, F_{}, F_{}, t, buf1, buf0, -1);
    }
    // the last MFMAs' results -> v_accvgpr_read (inline-asm MFMAs are not tracked by the
    // compiler's hazard recognizer)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#ifdef VP3D_ABLATION
    stamp(2);
    if (trc && tid == 0) trc[9] = mid_cyc;
#endif

    // the output resource starts at the tile's first row (outputs past 2^31 bytes: the
    // store offsets stay 32-bit and tile-relative; rows past M fall outside the range)
    const size_t y_rest = (size_t)(p.M - m0) * p.ldy * sizeof(CT);
    // ABL bit 3 (measurement): every store dropped by the range check (no output traffic)
    const __amdgpu_buffer_rsrc_t y_rsrc = make_rsrc(
        (const CT*)p.Y + (size_t)m0 * p.ldy, (ABL & 8) ? 0u : (uint32_t)(y_rest < 0x7FFFFFFFu ? y_rest : 0x7FFFFFFFu));
    if constexpr ((ABL & 16) != 0) {  // measurement: no epilogue at all (accumulators kept live)
#ifdef VP3D_ABLATION
        static_for<64>([&](auto r_c) __attribute__((always_inline)) {
            asm volatile("" ::"v"(aread<4 * decltype(r_c)::value>()));
        });
        if (ABL & 4) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            pinned_barrier();
            stamp(3);
        }
#endif
        return;
    }
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef int i32x2 __attribute__((ext_vector_type(2)));
    typedef short s16x2 __attribute__((ext_vector_type(2)));
    typedef CT ct2 __attribute__((ext_vector_type(2)));
    typedef CT ct4 __attribute__((ext_vector_type(4)));
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const int grp = lane >> 4;
    const int c0 = 8 * ((grp & 1) * 2 + (grp >> 1));
    // Packed epilogue (ReLU layers; the same bits as gemm::epilogue_tp): per 16 x 64 block the
    // 16 accumulators of a lane (channels nw + 16 j + 4 grp + 0..3 of one row) leave the AGPRs
    // and stay in accumulator layout: BN as v_pk_mul_f32 + v_pk_add_f32 (per element the two
    // roundings of x * scale + shift), with a residual (in LDS: read in accumulator layout,
    // 8 bytes per block) ReLU as an integer max on the f32 bits (negative and -0 -> +0, as
    // x > 0 ? x : 0) then the f32 add, one packed conversion per channel pair, without one
    // ReLU as an integer max on the packed 16-bit pair (the same bits: a pair's sign bit is
    // set exactly when ReLU-before-rounding gives +0); then one v_permlane16_swap per dword
    // pair gives each lane 8 consecutive channels for a 16-byte store (epilogue_tp: every
    // value in f32 through cmp/cndmask ReLU and an f32 swap -- 2.4x the instructions).
    auto epi_fast = [&](auto h_c, bool with_res) __attribute__((always_inline)) {
        constexpr int H = decltype(h_c)::value;
        const int nw = n0 + wc * 128 + 64 * H;
        f32x2 sc[4][2], sh[4][2];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = nw + 16 * j + 4 * grp;
            const f32x4 s4 = *(const f32x4*)&s_scale[n];
            const f32x4 h4 = *(const f32x4*)&s_shift[n];
            sc[j][0] = f32x2{s4[0], s4[1]};
            sc[j][1] = f32x2{s4[2], s4[3]};
            sh[j][0] = f32x2{h4[0], h4[1]};
            sh[j][1] = f32x2{h4[2], h4[3]};
        }
        // residual part H: row wr * 128 + 16 i + (lane & 15) of wave column wc, channel
        // 16 j + 4 grp at chunk 2 j + (grp >> 1) (swizzled), byte (grp & 1) * 8
        const char* rb = smem + ((nk - 2 + H) & 1) * GBUF + wc * 256 * 128 + wr * 128 * 128 + (lane & 15) * 128 +
                         (grp & 1) * 8;
        static_for<8>([&](auto i_c) __attribute__((always_inline)) {
            constexpr int I = decltype(i_c)::value;
            const int m = m0 + wr * 128 + 16 * I + (lane & 15);
            uint32_t pk[4][2];  // [block j][channel pair]
            static_for<4>([&](auto j_c) __attribute__((always_inline)) {
                constexpr int J = decltype(j_c)::value;
                constexpr int R = 4 * (8 * I + 4 * H + J);
                f32x2 v[2] = {f32x2{aread<R>(), aread<R + 1>()}, f32x2{aread<R + 2>(), aread<R + 3>()}};
                ct4 r4;
                if (with_res)
                    r4 = __builtin_bit_cast(
                        ct4, *(const u32x2*)(rb + I * 2048 + (((2 * J + (grp >> 1)) ^ fsw) << 4)));
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    f32x2 x = v[q] * sc[J][q];
                    x = x + sh[J][q];
                    if (with_res) {
                        i32x2 xi = __builtin_bit_cast(i32x2, x);
                        xi = __builtin_elementwise_max(xi, i32x2{0, 0});
                        x = __builtin_bit_cast(f32x2, xi);
                        x = x + f32x2{(float)r4[2 * q], (float)r4[2 * q + 1]};
                    }
                    s16x2 o = __builtin_bit_cast(s16x2, __builtin_convertvector(x, ct2));
                    if (!with_res) o = __builtin_elementwise_max(o, s16x2{0, 0});
                    pk[J][q] = __builtin_bit_cast(uint32_t, o);
                }
            });
            // the x dwords (blocks 0, 2) just written by VALU -> 2 wait states before the swap
            asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\tv_permlane16_swap_b32 %2, %3\n\t"
                         "v_permlane16_swap_b32 %4, %5\n\tv_permlane16_swap_b32 %6, %7"
                         : "+v"(pk[0][0]), "+v"(pk[1][0]), "+v"(pk[0][1]), "+v"(pk[1][1]), "+v"(pk[2][0]),
                           "+v"(pk[3][0]), "+v"(pk[2][1]), "+v"(pk[3][1]));
            const uint32_t yo =
                m < p.M ? (uint32_t)(((size_t)(m - m0) * p.ldy + nw + c0) * sizeof(CT)) : 0xFFFFFFC0u;
#pragma unroll
            for (int jp = 0; jp < 2; ++jp)
                __builtin_amdgcn_raw_buffer_store_b128(
                    u32x4{pk[2 * jp][0], pk[2 * jp][1], pk[2 * jp + 1][0], pk[2 * jp + 1][1]}, y_rsrc,
                    m < p.M ? yo + 64 * jp : 0xFFFFFFC0u, 0, 0);
        });
    };
    using H0 = std::integral_constant<int, 0>;
    using H1 = std::integral_constant<int, 1>;
    if (lres) {
        // part H landed: vmcnt(16) leaves in flight only younger pieces / stores (H = 0:
        // part 1's 16 pieces; H = 1: part 0's epilogue's 16 stores); then every wave's pieces
        // are visible after the barrier
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        pinned_barrier();
        epi_fast(H0{}, true);
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        pinned_barrier();
        epi_fast(H1{}, true);
    } else if (!p.R) {
        epi_fast(H0{}, false);
        epi_fast(H1{}, false);
    } else {  // residual with nk < 3: global loads row block by row block
        static_for<2>([&](auto h_c) __attribute__((always_inline)) {
            constexpr int H = decltype(h_c)::value;
            f32x4 acc[8][4];
            static_for<8>([&](auto i_c) __attribute__((always_inline)) {
                constexpr int I = decltype(i_c)::value;
                static_for<4>([&](auto j_c) __attribute__((always_inline)) {
                    constexpr int R = 4 * (8 * I + 4 * H + decltype(j_c)::value);
                    acc[I][decltype(j_c)::value] = f32x4{aread<R>(), aread<R + 1>(), aread<R + 2>(), aread<R + 3>()};
                });
            });
            epilogue_tp<CT, 8, false, 1, 0>(p, acc, m0 + wr * 128, n0 + wc * 128 + 64 * H, lane, s_scale, s_shift,
                                            y_rsrc, nullptr, m0);
        });
    }
#ifdef VP3D_ABLATION
    if (ABL & 4) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        pinned_barrier();
        stamp(3);
    }
#endif
}

#undef A4_C10
#undef A4_ALL_AGPRS

}  // namespace

#ifdef VP3D_ABLATION
hipError_t conv_gemm_a4_set_trace(unsigned long long* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_a4_trace), &buf, sizeof(buf));
}
#endif

bool conv_gemm_a4_eligible(const ConvGemmParams& p, Act a_type, Act out_type, Act compute) {
    if (compute == Act::F32 || a_type != compute || out_type != compute) return false;
    if (p.relu != 1) return false;  // the packed epilogue is the BN + ReLU one
    if (p.Ktap % GK != 0 || p.Kp % GK != 0 || p.lda % 8 != 0) return false;
    if (p.N % GN != 0 || p.N > GMAXN || p.ldy % 8 != 0 || (p.R && p.ldr % 8 != 0)) return false;
    if ((reinterpret_cast<uintptr_t>(p.A) & 15) || (reinterpret_cast<uintptr_t>(p.Y) & 15) ||
        (p.R && (reinterpret_cast<uintptr_t>(p.R) & 15)))
        return false;
    return (size_t)p.N * p.Kp < (1u << 31);
}

hipError_t launch_conv_gemm_a4(const ConvGemmParams& p, Act compute, hipStream_t stream) {
    const dim3 grid(((p.M + GM - 1) / GM) * (p.N / GN));
#ifdef VP3D_ABLATION
    // measurement builds only (tools/ubench/gemm_check): VP3D_ABL=1 no loop DMA, 2 no loop
    // fragment reads, 3 neither (wrong results, timing only)
    static const int abl = [] {
        const char* e = getenv("VP3D_ABL");
        return e ? atoi(e) : 0;
    }();
    if (compute == Act::BF16 && abl >= 1) {
        switch (abl) {
            case 1: hipLaunchKernelGGL((conv_gemm_a4<__bf16, 1>), grid, dim3(256), 0, stream, p); break;
            case 2: hipLaunchKernelGGL((conv_gemm_a4<__bf16, 2>), grid, dim3(256), 0, stream, p); break;
            case 3: hipLaunchKernelGGL((conv_gemm_a4<__bf16, 3>), grid, dim3(256), 0, stream, p); break;
            case 4: hipLaunchKernelGGL((conv_gemm_a4<__bf16, 4>), grid, dim3(256), 0, stream, p); break;
            case 8: hipLaunchKernelGGL((conv_gemm_a4<__bf16, 8>), grid, dim3(256), 0, stream, p); break;
            case 12: hipLaunchKernelGGL((conv_gemm_a4<__bf16, 12>), grid, dim3(256), 0, stream, p); break;
            case 16: hipLaunchKernelGGL((conv_gemm_a4<__bf16, 16>), grid, dim3(256), 0, stream, p); break;
            default: hipLaunchKernelGGL((conv_gemm_a4<__bf16, 20>), grid, dim3(256), 0, stream, p); break;
        }
        return hipGetLastError();
    }
#endif
    if (compute == Act::BF16)
        hipLaunchKernelGGL((conv_gemm_a4<__bf16, 0>), grid, dim3(256), 0, stream, p);
    else
        hipLaunchKernelGGL((conv_gemm_a4<_Float16, 0>), grid, dim3(256), 0, stream, p);
    return hipGetLastError();
}

}  // namespace vp3d
