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
constexpr int kVm32Lgkm0 = 0x8070; // vmcnt(32) lgkmcnt(0)

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

#ifdef VP3D_ABLATION
// measurement builds (ABL bit 6): a[R..R+15] (+)= one v_mfma_f32_32x32x16 on the same fragment
// registers -- the issue pattern of a 32 x 32 block K loop (results wrong; timing only)
template <typename CT, int R, bool ZERO>
__device__ __forceinline__ void amma32(const u32x4& w, const u32x4& a) {
    if constexpr (std::is_same<CT, __bf16>::value) {
        if constexpr (ZERO)
            asm volatile("v_mfma_f32_32x32x16_bf16 a[%c2:%c3], %0, %1, 0" ::"v"(w), "v"(a), "i"(R), "i"(R + 15));
        else
            asm volatile("v_mfma_f32_32x32x16_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(w), "v"(a), "i"(R),
                         "i"(R + 15));
    } else {
        if constexpr (ZERO)
            asm volatile("v_mfma_f32_32x32x16_f16 a[%c2:%c3], %0, %1, 0" ::"v"(w), "v"(a), "i"(R), "i"(R + 15));
        else
            asm volatile("v_mfma_f32_32x32x16_f16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(w), "v"(a), "i"(R),
                         "i"(R + 15));
    }
}
#endif

// an empty asm on a wave-uniform value: the compiler can no longer see through it (no
// hoisting or precomputing of what derives from it)
__device__ __forceinline__ void launder_s(int& x) { asm volatile("" : "+s"(x)); }
__device__ __forceinline__ void launder_lane_consts(int& a, int& b, int& c, int& d, int& e, int& f, int& g, int& h,
                                                    int& i) {
    asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h), "+v"(i));
}
// (inline asm with operand constraints lives in __device__ helpers: in a kernel body the host
// compilation rejects the AMDGPU constraints silently and emits no launch stub)
__device__ __forceinline__ void launder_params(ConvGemmParams& p) {
    asm volatile("" : "+s"(p.M), "+s"(p.Kp), "+s"(p.T_out), "+s"(p.T_in), "+s"(p.stride), "+s"(p.dil), "+s"(p.Ktap),
                 "+s"(p.lda), "+s"(p.R_T), "+s"(p.R_stride), "+s"(p.R_off), "+s"(p.ldr), "+s"(p.ldy));
    asm volatile("" : "+s"(p.A), "+s"(p.W), "+s"(p.R), "+s"(p.Y));
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

// HN (half-N tiles, a launch's partial last round): 256 x 128 tiles -- each wave 128 rows x 64
// channels, accumulator blocks (i, j < 4), 8 A + 4 W LDS-DMA pieces per K-tile -- over the
// M-tiles from p.sk_full on, one unit per workgroup (no walk, no split, no residual).  Every
// output keeps the whole tile's K order, so the same bits as a 256 x 256 tile.
// HNL = 2 (quarter-N, f16x3 only): 256 x 64 tiles, each wave 128 x 32, for tails of <= a
// quarter round.
template <typename CT, int ABL, int X3 = 0, bool GD = true, bool SPLIT = false, int HNL = 0>
__global__ __launch_bounds__(256, 1) void conv_gemm_a4(ConvGemmParams p_arg) {
    constexpr bool HN = HNL > 0;
    static_assert(!HN || (GD && !SPLIT), "half-N tiles: grouped pieces, no split");
    static_assert(HNL < 2 || X3 != 0, "quarter-N tiles: the split-fp16 epilogue only");
    constexpr int TN = GN >> HNL;  // tile channels
    constexpr int NJ = TN / 32;    // channel blocks of 16 per wave (two wave columns)
    constexpr int WP = TN / 32;    // W pieces per wave and K-tile (TN rows x 128 B, 4 waves)
    constexpr int NB = NJ < 4 ? NJ : 4;  // blocks of a 64-channel epilogue half
    // the accumulator file is this kernel's own from here on (see the header)
    asm volatile("" ::: A4_ALL_AGPRS);
    // a copy whose fields go through an empty asm every tile (below): values derived from them
    // are then recomputed per tile instead of hoisted out of the tile loop and kept live
    ConvGemmParams p = p_arg;

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

    const int ntn = p.N / TN;
    const int ntm = (p.M + GM - 1) / GM;
    const int mt_base = HN ? p.sk_full : 0;  // HN: the first M-tile of the launch
    const int ntiles = (ntm - mt_base) * ntn;
    const int nk_all = p.Kp / GK;  // >= 1
    // Work units: tile u < sk_full whole; with a split plan (ConvGemmParams::sk_*) the sk_left
    // tiles after them as S units each -- unit full + v: tile full + v % L, K range q = S - 1 -
    // v / L (helpers first, the owner q = 0 dispatched last: the owners wait for their helpers,
    // which never wait).  Per unit: kb / nk (first K-tile, K-tiles), role, the tile's slot.
    const int S = SPLIT ? p.sk_split : 1;  // SPLIT launches only (no split code otherwise)
    const int sk_full = S > 1 ? p.sk_full : ntiles;
    const int nunits = S > 1 ? sk_full + S * p.sk_left : ntiles;
    constexpr int kWhole = 0, kOwner = 1, kHelper = 2;
    int kb = 0, nk = nk_all, role = kWhole, sidx = 0, sq = 0;
    // 1x1 convs (residual): the tile's residual rows land in LDS by LDS-DMA during the last
    // two K-tiles, into the operand buffers those no longer need -- part h (the channel half
    // h of both wave columns: 256 rows x 2 x 128 B = 64 KiB) in phase B of tile nk - 2 + h,
    // in the DMA slots; rows at 128-byte pitch with the operands' chunk swizzle -- so the
    // epilogue reads them from LDS instead of waiting on global loads row block by row block
    const bool lres_layer = X3 == 0 && p.R != nullptr && nk_all >= 3;
    bool lres = lres_layer;  // per unit: helpers run no epilogue
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

    // ---- per-tile operand addressing.  DMA pieces: 8 rows x 128 B each, 32 per operand;
    // wave w issues q = w + 4 i.  Lane l fills row 8q + (l >> 3), physical chunk (l & 7) =
    // logical chunk lc ^ swz; all pieces of a wave share the parity of q (= that of w): one
    // swizzled chunk each.  LDS-DMA as buffer_load ... lds through per-tile resources: 32-bit
    // lane offsets fixed for the tile, the K-tile's k offset in soffset, so no per-piece address
    // arithmetic (global_load_lds from 64-bit lane pointers measured 2 % slower: block-1 k3
    // shape, B = 8192, 1.251-1.262 vs 1.231-1.237 ms) ----
    int prow = lane >> 3;
    int lc = (lane & 7) ^ (((wid & 1) * 4 + (prow >> 1)) & 7);
    // GD (grouped pieces): wave w's 8 A pieces are the consecutive slots 8w .. 8w + 7 (tile rows
    // 64w .. 64w + 63; W likewise), issued as 2 groups of 4 that share one LDS base (M0) and
    // differ by the instruction offset (i & 3) KiB -- applied to the LDS and the global address
    // alike, so the lane offsets carry - (i & 3) KiB against resources based 3 KiB early.  One
    // M0 write per 4 pieces instead of one per piece.  Otherwise slot w + 4i, M0 per piece.
    constexpr int kReb = GD ? 3072 : 0;
    int m0 = 0, n0 = 0;
    uint32_t va[8], vw[8], vr[8];
    __amdgpu_buffer_rsrc_t a_rsrc, w_rsrc, r_rsrc;
    auto setup = [&](int unit) __attribute__((always_inline)) {
        int tix = unit;
        kb = 0;
        nk = nk_all;
        role = kWhole;
        if (S > 1 && unit >= sk_full) {
            const int v = unit - sk_full;
            sidx = v % p.sk_left;
            sq = S - 1 - v / p.sk_left;
            tix = sk_full + sidx;
            kb = sq * (nk_all / S);
            nk = nk_all / S;
            role = sq == 0 ? kOwner : kHelper;
        }
        lres = lres_layer && role != kHelper && nk >= 3;
        const int wg = xcd_remap(tix, ntiles);
        const int tile_m = wg / ntn;
        const int tile_n = wg - tile_m * ntn;
        m0 = (mt_base + tile_m) * GM;
        n0 = tile_n * TN;
        const int srow0 = src_row(p, m0);  // m0 < M; wave-uniform
        a_rsrc = make_rsrc((const char*)((const CT*)p.A + (int64_t)srow0 * p.lda) - kReb, 0x7FFFFFFFu);
        w_rsrc = make_rsrc((const char*)((const CT*)p.W + (int64_t)n0 * p.Kp) - kReb, 0x7FFFFFFFu);
        const int rrow0 = lres ? res_row(p, m0) : 0;
        r_rsrc = make_rsrc((const char*)(lres ? (const CT*)p.R + (int64_t)rrow0 * p.ldr : (const CT*)p.A) - kReb,
                           0x7FFFFFFFu);
        // lane values from a fresh laundered copy: nothing setup derives from them is computed
        // ahead of the call and kept live across a K loop or an epilogue
        int sln = lane, swv = widu;
        asm volatile("" : "+v"(sln));
        launder_s(swv);
        const int spr = sln >> 3;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int q = GD ? 8 * swv + i : swv + 4 * i;  // the piece's slot: rows 8q .. 8q + 7
            const int qw = HN ? WP * swv + (i % WP) : q;   // HN: WP W slots per wave
            const int lci = GD ? (sln & 7) ^ (((i & 1) * 4 + (spr >> 1)) & 7) : lc;
            const int reb = GD ? kReb - (i & 3) * 1024 : 0;
            int m = m0 + 8 * q + spr;
            m = m < p.M ? m : p.M - 1;  // rows past M read a valid row; never stored
            va[i] = (uint32_t)(((src_row(p, m) - srow0) * p.lda + lci * 8) * (int)sizeof(CT) + reb);
            vw[i] = (uint32_t)(((8 * qw + prow) * p.Kp + lci * 8) * (int)sizeof(CT) + reb);  // W rows padded
            vr[i] = lres ? (uint32_t)(((res_row(p, m) - rrow0) * p.ldr + lci * 8) * (int)sizeof(CT) + reb) : 0u;
        }
    };
    // piece k of residual part h: wave column k >> 3, the rows of A piece k & 7
    // LDS-DMA destination of piece slot `q` (of 64 per 64 KiB region) in `buf`: the wave id goes
    // through an empty asm at every use, so each destination is one scalar add at its
    // issue instead of 64 precomputed SGPRs kept live across the tile loop
    auto lds_dst = [&](char* buf, int q) __attribute__((always_inline)) -> char* {
        int w = widu;
        launder_s(w);
        return buf + (w + q) * 1024;
    };
    // GD: the LDS bases (M0) of this wave's piece groups in a 64 KiB buffer -- A pieces 0-3, 4-7,
    // W pieces 0-3, 4-7 -- computed once per phase (one laundered wave id), so the compiler can
    // keep M0 across a group's 4 pieces
    struct Bases {
        char* g[4];
    };
    auto bases_of = [&](char* buf) __attribute__((always_inline)) -> Bases {
        int w = widu;
        launder_s(w);
        char* b = buf + 8 * w * 1024;
        if constexpr (HN) return Bases{{b, b + 4096, buf + GW_OFF + WP * w * 1024, nullptr}};
        return Bases{{b, b + 4096, b + GW_OFF, b + GW_OFF + 4096}};
    };
    auto piece_lds = [&](char* buf, int i) __attribute__((always_inline)) -> char* {
        if constexpr (GD) {
            int w = widu;
            launder_s(w);
            return buf + (8 * w + (i & 4)) * 1024;
        } else {
            return lds_dst(buf, 4 * i);
        }
    };
    // (piece indices as integral constants: the instruction offset is an immediate)
    auto res_piece = [&](char* buf, auto k_c, int h) __attribute__((always_inline)) {
        constexpr int k = decltype(k_c)::value;
        constexpr int wcp = k >> 3;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r_rsrc, (lds_ptr_t)piece_lds(buf + wcp * 32 * 1024, k & 7), 16,
                                                 vr[k & 7], (uint32_t)((n0 + 128 * wcp + 64 * h) * (int)sizeof(CT)),
                                                 GD ? (k & 3) * 1024 : 0, 0);
    };
    // k offset of K-tile s inside a row: tap * dil rows + channel base (wave-uniform)
    auto a_koff = [&](int s) __attribute__((always_inline)) -> int64_t {
        const int k0 = (kb + s) * GK;
        const int tap = k0 / p.Ktap;
        return (int64_t)tap * p.dil * p.lda + (k0 - tap * p.Ktap);
    };
    auto dma_piece = [&](char* buf, auto i_c, int s, int64_t aoff, const Bases& bs) __attribute__((always_inline)) {
        constexpr int i = decltype(i_c)::value;
        char* const ldsp = GD ? bs.g[i >> 2] : (i < 8 ? lds_dst(buf, 4 * i) : lds_dst(buf + GW_OFF, 4 * (i - 8)));
        if constexpr (i < 8)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, (lds_ptr_t)ldsp, 16, va[i],
                                                     (uint32_t)aoff * (uint32_t)sizeof(CT), GD ? (i & 3) * 1024 : 0, 0);
        else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(w_rsrc, (lds_ptr_t)ldsp, 16, vw[i - 8],
                                                     (uint32_t)((kb + s) * GK * (int)sizeof(CT)), GD ? (i & 3) * 1024 : 0, 0);
    };
    char* const buf0 = smem;
    char* const buf1 = smem + GBUF;
    // K-tiles 0 and 1 of the current tile into buffers 0 and 1
    auto stage_01 = [&]() __attribute__((always_inline)) {
        const int64_t o0 = a_koff(0);
        const Bases b0 = bases_of(buf0);
        static_for<8 + WP>([&](auto i_c) __attribute__((always_inline)) { dma_piece(buf0, i_c, 0, o0, b0); });
        if (nk > 1) {
            const int64_t o1 = a_koff(1);
            const Bases b1 = bases_of(buf1);
            static_for<8 + WP>([&](auto i_c) __attribute__((always_inline)) { dma_piece(buf1, i_c, 1, o1, b1); });
        }
    };

    // ---- fragment reads (q64's layout): row (l & 15) of a 16-row block, logical chunk
    // 4 kh + (l >> 4), physical chunk ^ ((l & 15) >> 1) ----
    int fsw = (lane & 15) >> 1;
    int fo0 = (lane & 15) * 128 + (((lane >> 4) ^ fsw) << 4);
    int fo1 = (lane & 15) * 128 + ((((lane >> 4) + 4) ^ fsw) << 4);
    int a_base = wr * 128 * 128;
    int w_base = GW_OFF + wc * (TN / 2) * 128;

    u32x4 fa[2][8], fw[2][8];  // [set][block]

    // 64 MFMAs on set CUR; RD: the 16 reads of set NXT from `rbuf` at k-half offset `fo`;
    // DMA: the 16 pieces of K-tile `s` into `dbuf`, two per row block; otherwise resp >= 0:
    // residual part resp into `dbuf` in the same slots
    auto phase = [&](auto cur_c, auto zero_c, auto rd_c, auto dma_c, const char* rbuf, int fo, char* dbuf, int s,
                     int resp) __attribute__((always_inline)) {
        constexpr int CUR = decltype(cur_c)::value;
        constexpr int NXT = CUR ^ 1;
        constexpr bool ZERO = decltype(zero_c)::value;
        constexpr bool RD = decltype(rd_c)::value;
        constexpr bool DMA = decltype(dma_c)::value;
        const int64_t aoff = DMA ? a_koff(s) : 0;
        const Bases bs = DMA ? bases_of(dbuf) : Bases{};
        // each row block: the MFMA on channel block j, with one memory instruction ahead of
        // the even ones: A read, DMA piece, W read, DMA piece (bursts of 2 reads + 2 pieces
        // at the row block's start measured 3 % slower at B = 8192, the same at 65,536;
        // 4 pieces in each of the first 4 row blocks 3-6 % slower).  ABL (measurement
        // builds): bit 0 no loop DMA, bit 1 no loop fragment reads
        constexpr bool DO_RD = RD && !(ABL & 2);
        constexpr bool DO_DMA = DMA && !(ABL & 1);
#ifdef VP3D_ABLATION
        if constexpr ((ABL & 64) != 0 && !HN) {
            // 32 x 32 blocks: 16 blocks x 2 k-steps of 16, one memory instruction ahead of each
            // MFMA (the 16 reads on the even ones, the 16 DMA pieces on the odd ones)
            static_for<32>([&](auto n_c) __attribute__((always_inline)) {
                constexpr int n = decltype(n_c)::value;
                constexpr int b = n >> 1, ks = n & 1, h = n >> 1;
                if constexpr (DO_RD && (n & 1) == 0) {
                    if constexpr (h < 8)
                        fa[NXT][h] = *(const u32x4*)(rbuf + a_base + h * 2048 + fo);
                    else
                        fw[NXT][h - 8] = *(const u32x4*)(rbuf + w_base + (h - 8) * 2048 + fo);
                }
                if constexpr (DO_DMA && (n & 1) == 1) dma_piece(dbuf, std::integral_constant<int, h>{}, s, aoff, bs);
                if constexpr (!DMA && (n & 1) == 1) {
                    if (resp >= 0) res_piece(dbuf, std::integral_constant<int, h>{}, resp);
                }
                amma32<CT, 16 * b, ZERO>(fw[CUR][(b & 3) * 2 + ks], fa[CUR][(b >> 2) * 2 + ks]);
                __builtin_amdgcn_sched_barrier(0);
            });
            if constexpr (RD) __builtin_amdgcn_s_waitcnt(kLgkm0);
            return;
        }
#endif
        static_for<8>([&](auto i_c) __attribute__((always_inline)) {
            constexpr int I = decltype(i_c)::value;
            static_for<NJ>([&](auto j_c) __attribute__((always_inline)) {
                constexpr int J = decltype(j_c)::value;
                if constexpr (HN) {
                    // NJ MFMAs per row block: A read, DMA piece I (A), W read (I < NJ), piece 8 + I (W)
                    constexpr int JWR = NJ > 2 ? 2 : 1;
                    if constexpr (DO_RD && J == 0) fa[NXT][I] = *(const u32x4*)(rbuf + a_base + I * 2048 + fo);
                    if constexpr (DO_DMA && J == 1) dma_piece(dbuf, std::integral_constant<int, I>{}, s, aoff, bs);
                    if constexpr (DO_RD && J == JWR && I < NJ)
                        fw[NXT][I] = *(const u32x4*)(rbuf + w_base + I * 2048 + fo);
                    if constexpr (DO_DMA && J == NJ - 1 && I < WP)
                        dma_piece(dbuf, std::integral_constant<int, 8 + I>{}, s, aoff, bs);
                } else {
                    if constexpr (DO_RD && J == 0) fa[NXT][I] = *(const u32x4*)(rbuf + a_base + I * 2048 + fo);
                    if constexpr (DO_RD && J == 4) fw[NXT][I] = *(const u32x4*)(rbuf + w_base + I * 2048 + fo);
                    if constexpr (DO_DMA && (J == 2 || J == 6))
                        dma_piece(dbuf, std::integral_constant<int, 2 * I + J / 4>{}, s, aoff, bs);
                    if constexpr (!DMA && (J == 2 || J == 6)) {
                        if (resp >= 0) res_piece(dbuf, std::integral_constant<int, 2 * I + J / 4>{}, resp);
                    }
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

    // the wait before a K-tile's phase B: vm = 0 all operand pieces landed; 16: the 16
    // residual pieces of part 0 (issued in the phase before) may stay in flight; 32: the
    // previous tile's 32 epilogue stores (younger than this tile's first two K-tiles) may
    auto mid = [&](int vm) __attribute__((always_inline)) {
#ifdef VP3D_ABLATION
        const unsigned long long c0 = (ABL & 4) ? __builtin_amdgcn_s_memtime() : 0;
#endif
        if (vm == 16)
            __builtin_amdgcn_s_waitcnt(kVm16Lgkm0);
        else if (vm == 32)
            __builtin_amdgcn_s_waitcnt(kVm32Lgkm0);
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
    // K-tile t in buffer `b` (the other one `o`); RD / DMA: K-tile t + 1 / t + 2 exists;
    // resp >= 0: residual part resp into `b` in phase B
    auto ktile = [&](auto zero_c, auto rd_c, auto dma_c, int t, char* b, char* o, int resp, int vm) __attribute__((always_inline)) {
        phase(C0{}, zero_c, T_{}, F_{}, b, fo1, nullptr, 0, -1);
        mid(vm);
        phase(C1{}, F_{}, rd_c, dma_c, o, fo0, b, t + 2, resp);
    };

    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef int i32x2 __attribute__((ext_vector_type(2)));
    typedef short s16x2 __attribute__((ext_vector_type(2)));
    typedef CT ct2 __attribute__((ext_vector_type(2)));
    typedef CT ct4 __attribute__((ext_vector_type(4)));
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    int grp = lane >> 4;
    int c0 = 8 * ((grp & 1) * 2 + (grp >> 1));
    // Packed epilogue (ReLU layers; the same bits as gemm::epilogue_tp): per 16 x 64 block the
    // 16 accumulators of a lane (channels nw + 16 j + 4 grp + 0..3 of one row) leave the AGPRs
    // and stay in accumulator layout: BN as v_pk_mul_f32 + v_pk_add_f32 (per element the two
    // roundings of x * scale + shift), with a residual (read from LDS into registers in
    // accumulator layout, 8 bytes per block) ReLU as an integer max on the f32 bits (negative
    // and -0 -> +0, as x > 0 ? x : 0) then the f32 add, one packed conversion per channel pair,
    // without one ReLU as an integer max on the packed 16-bit pair (the same bits: a pair's
    // sign bit is set exactly when ReLU-before-rounding gives +0); then one v_permlane16_swap
    // per dword pair gives each lane 8 consecutive channels for a 16-byte store
    // (epilogue_tp: every value in f32 through cmp/cndmask ReLU and an f32 swap -- 2.4x the
    // instructions).  em0 / en0: the tile's origin (m0 / n0 may already be the next tile's).
    // a residual part in registers (accumulator layout), so its buffer can take one of the
    // next tile's first two K-tiles before that half's stores
    u32x2 resr[8][4];
    int enk = nk;  // the K-tiles of the unit whose epilogue runs (the next unit's setup may be done)
    auto res_addr = [&](int h, int i, int j) __attribute__((always_inline)) -> const u32x2* {
        return (const u32x2*)(smem + ((enk - 2 + h) & 1) * GBUF + wc * 256 * 128 + wr * 128 * 128 + (lane & 15) * 128 +
                              (grp & 1) * 8 + i * 2048 + (((2 * j + (grp >> 1)) ^ fsw) << 4));
    };
    // ---- split-K partial sums: a helper unit stores its 256 accumulators per lane (64 x 16 B,
    // [wave][block / 4][lane] in its 256 KiB slot: whole 1 KiB runs per instruction), releases
    // them at agent scope (the owner may sit on another XCD) and counts itself in the tile's
    // flag; the owner waits for S - 1 (bounded: 1 s, never expected), acquires, and adds the
    // helpers' values to its own, in unit order, as it reads its accumulators ----
    auto part_ptr = [&](int si, int q) __attribute__((always_inline)) -> float* {
        return p.sk_part + (size_t)(si * (S - 1) + (q - 1)) * 65536 + (size_t)wid * 16384 + lane * 4;
    };
    auto helper_store = [&](int si, int q) __attribute__((always_inline)) {
        float* const base = part_ptr(si, q);
        static_for<64>([&](auto r_c) __attribute__((always_inline)) {
            constexpr int R4 = decltype(r_c)::value;
            *(f32x4*)(base + R4 * 256) = f32x4{aread<4 * R4>(), aread<4 * R4 + 1>(), aread<4 * R4 + 2>(), aread<4 * R4 + 3>()};
        });
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        pinned_barrier();
        if (tid == 0) {
            const SplitCtl* ctl = (const SplitCtl*)((const char*)p.sk_flag + kSplitCtlOffset);
            if (!ctl->drop) __hip_atomic_fetch_add(p.sk_flag + si, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    // bounded (SplitCtl::spin_ticks); on the bound the fault goes to the host-mapped word and
    // the epilogue runs on (its output is reported wrong by the host, vp3d_sync_status)
    auto owner_wait = [&](int si) __attribute__((always_inline)) {
        if (tid == 0) {
            const SplitCtl* ctl = (const SplitCtl*)((const char*)p.sk_flag + kSplitCtlOffset);
            const unsigned long long spin = ctl->spin_ticks;
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(p.sk_flag + si, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < S - 1) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > spin) {
                    unsigned* err = ctl->err;
                    if (err) __hip_atomic_fetch_or(err, kFaultSplitTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
            }
        }
        pinned_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    };
    // v (the accumulators of block R as two pairs) += the helpers' values of that block
    auto owner_add = [&](auto r_c, int si, f32x2 (&v)[2]) __attribute__((always_inline)) {
        constexpr int R = decltype(r_c)::value;
        for (int q = 1; q < S; ++q) {
            const f32x4 pr = *(const f32x4*)(part_ptr(si, q) + (R / 4) * 256);
            v[0] = v[0] + f32x2{pr[0], pr[1]};
            v[1] = v[1] + f32x2{pr[2], pr[3]};
        }
    };
    auto owner_done = [&](int si) __attribute__((always_inline)) {
        if (tid == 0) __hip_atomic_fetch_sub(p.sk_flag + si, S - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto epi_fast = [&](auto h_c, bool with_res, int em0, int en0, __amdgpu_buffer_rsrc_t y_rsrc, int own_si) __attribute__((always_inline)) {
        constexpr int H = decltype(h_c)::value;
        const int nw = en0 + wc * (TN / 2) + 64 * H;
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
        static_for<8>([&](auto i_c) __attribute__((always_inline)) {
            constexpr int I = decltype(i_c)::value;
            const int m = em0 + wr * 128 + 16 * I + (lane & 15);
            uint32_t pk[4][2];  // [block j][channel pair]
            static_for<4>([&](auto j_c) __attribute__((always_inline)) {
                constexpr int J = decltype(j_c)::value;
                constexpr int R = 4 * (8 * I + 4 * H + J);
                f32x2 v[2] = {f32x2{aread<R>(), aread<R + 1>()}, f32x2{aread<R + 2>(), aread<R + 3>()}};
                if (own_si >= 0) owner_add(std::integral_constant<int, R>{}, own_si, v);
                ct4 r4;
                if (with_res) r4 = __builtin_bit_cast(ct4, resr[I][J]);
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
            const uint32_t yo = (uint32_t)(((size_t)(m - em0) * p.ldy + nw + c0) * sizeof(CT));
#pragma unroll
            for (int jp = 0; jp < 2; ++jp)
                __builtin_amdgcn_raw_buffer_store_b128(
                    u32x4{pk[2 * jp][0], pk[2 * jp][1], pk[2 * jp + 1][0], pk[2 * jp + 1][1]}, y_rsrc,
                    m < p.M ? yo + 64 * jp : 0xFFFFFFC0u, 0, 0);
        });
    };
    using H0 = std::integral_constant<int, 0>;
    using H1 = std::integral_constant<int, 1>;
    int res0 = -1, res1 = -1;  // per unit (below)

    // ---- the tiles of this workgroup: blockIdx.x, + gridDim.x, ... (a grid of one
    // workgroup per CU walks them; with one tile per workgroup the loop runs once).  The
    // next tile's K-tiles 0 and 1 are staged before this tile's epilogue stores (without a
    // residual in phase B of the last K-tile; with one once the residual is in registers),
    // so its first waits leave the stores in flight (vmcnt counts in issue order) ----
    int tix = blockIdx.x;
    setup(tix);
    stage_01();
    bool first = true;
    bool prev_lres = false;  // the previous unit's epilogue took residual parts (its store order)
    bool x3_prev_res = false;  // X3: the previous unit's epilogue loaded residual rows after its DMA
    bool x3_prev_xres = false;  // X3: ... took its residual through LDS (K-tiles 0, 1 issued before its H1 stores)
    for (;;) {
        // the per-lane constants go through an empty asm every tile: otherwise the compiler
        // hoists every address derived from them out of the tile loop and keeps them live
        // across it (past 256 VGPRs, into the accumulator file)
        launder_lane_consts(prow, lc, fsw, fo0, fo1, a_base, w_base, grp, c0);
        launder_params(p);
        const int next = HN ? nunits : tix + (int)gridDim.x;  // (HN: one unit per workgroup)
        const bool has_next = next < nunits;
        res0 = lres ? 0 : -1;
        res1 = lres ? 1 : -1;
        if (first) {
            if (nk > 1)
            {
                if constexpr (HN)
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 + WP) : "memory");  // K-tile 0 landed (younger: K-tile 1)
                else
                    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            }
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // scale / shift stores
        } else if constexpr (X3 != 0) {
            // with a residual nothing to wait for: K-tiles 0 and 1 were issued before the
            // previous epilogue's residual loads, which it waited for (vmcnt retires in issue
            // order); only its last stores may still be in flight.  Without one (a walked layer
            // with no residual: VP3D_A4_WALK=2; a helper unit's release fence drained anyway)
            // they may not have landed: drain.
            // with the residual through LDS: K-tile 0 landed; younger are K-tile 1 and the previous
            // epilogue's 32 H1 stores
            if (x3_prev_xres)
                asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
            else if (!x3_prev_res)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            // younger: K-tile 1 (16 pieces) and the previous epilogue's 32 stores (with a
            // residual: the H0 stores, K-tile 1, the H1 stores)
            asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
        }
        pinned_barrier();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            fa[0][i] = *(const u32x4*)(buf0 + a_base + i * 2048 + fo0);
            if (i < NJ) fw[0][i] = *(const u32x4*)(buf0 + w_base + i * 2048 + fo0);
        }
        if constexpr (X3 != 0) {
            // ---- split fp16 (VP3D_DTYPE_F16X3): rows hold every f32 value as f16 halves, each
            // 32-wide K group [hi(32) | lo(32)], so a 64-deep K-tile carries 32 K values: its
            // k 0..31 fragments are the hi halves, k 32..63 the lo ones.  Per K-tile and
            // accumulator, in q64's order (the same bits): W_hi.A_hi, W_hi.A_lo, W_lo.A_hi
            // (the lo.lo term, 2^-22 relative, dropped).  W_hi / W_lo stay in fw[0] / fw[1];
            // A_hi of K-tile t sits in fa[t & 1], A_lo in the other set:
            //   A  (64 MFMAs W_hi.A_hi):  reads W_lo -> fw[1], A_lo -> fa[1-h]      (K-tile t)
            //   mid: vmcnt(0), lgkmcnt(0), barrier
            //   B1 (64 MFMAs W_hi.A_lo):  A_hi of t + 1 -> fa[1-h], row block i-1 in row block i
            //                             (its A_lo used up); 8 DMA pieces of t + 2
            //   B2 (64 MFMAs W_lo.A_hi):  W_hi of t + 1 -> fw[0] (used up in B1); 8 DMA pieces
            // ---- the 1x1 + residual layers: the residual through LDS (round 5).  A tile's residual
            // is 256 rows x 256 channels of [hi | lo] halves = 256 KiB: four quarters Q(hh, wc) of
            // 64 KiB (channel half hh of wave column wc: 256 rows x 256 contiguous bytes, two groups
            // of 32 channels, [hi | lo] each).  Q(0, 0) and Q(0, 1) land by LDS-DMA in phase B of
            // the last two K-tiles (their own buffers, which no later K-tile needs), Q(1, *) during
            // the half-0 epilogue; the next tile's K-tiles 0 and 1 are staged once half 1 is read.
            // LDS image: 1 KiB slot 2q + s = rows 8q .. 8q + 7 (q = the A piece of those rows), the
            // 128-byte group s of each row, 16-byte chunks with the A pieces' swizzle.  Per-lane
            // source offsets vr[i] (the A pieces' rows, computed once the A / W DMA offsets are
            // dead: the K loop has no VGPRs to spare) ----
            const bool xres = X3 == 1 && !SPLIT && !HN && !(ABL & 40) && p.R != nullptr && role != kHelper && nk >= 3;
            __amdgpu_buffer_rsrc_t xr_rsrc;
            auto xres_prep = [&]() __attribute__((always_inline)) {
                // lane values through an empty asm: nothing derived from them is hoisted out of
                // the tile loop (the K loop has no VGPRs to spare)
                int ln = lane, wv = widu;
                asm volatile("" : "+v"(ln));
                launder_s(wv);
                const int pr = ln >> 3;
                const int rrow0x = res_row(p, m0);
                xr_rsrc = make_rsrc((const char*)((const f16*)p.R + (int64_t)rrow0x * p.ldr), 0x7FFFFFFFu);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    int m = m0 + 8 * (8 * wv + i) + pr;
                    m = m < p.M ? m : p.M - 1;
                    const int lci = (ln & 7) ^ (((i & 1) * 4 + (pr >> 1)) & 7);
                    vr[i] = (uint32_t)((res_row(p, m) - rrow0x) * p.ldr * 2 + lci * 16);
                }
            };
            // piece (i, s) of quarter (hh, wcq): this wave's A-piece rows i, 128-byte group s
            auto xres_piece = [&](char* buf, auto i_c, auto s_c, int wcq, int hh) __attribute__((always_inline)) {
                constexpr int I = decltype(i_c)::value;
                constexpr int S2 = decltype(s_c)::value;
                int w = widu;
                launder_s(w);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(xr_rsrc, (lds_ptr_t)(buf + (2 * (8 * w + I) + S2) * 1024), 16, vr[I],
                                                         (uint32_t)(4 * (n0 + wcq * 128 + 64 * hh) + S2 * 128), 0, 0);
            };
            auto x3_phase = [&](auto h_c, auto kind_c, auto zero_c, auto rd_c, auto dma_c, const char* rbuf, char* dbuf,
                                int s, auto rq_c, char* rqbuf) __attribute__((always_inline)) {
                constexpr int RQ = decltype(rq_c)::value;  // residual quarter (0, RQ) into rqbuf, or -1
                constexpr int H = decltype(h_c)::value;
                constexpr int KIND = decltype(kind_c)::value;  // 0 = A, 1 = B1, 2 = B2
                constexpr bool ZERO = decltype(zero_c)::value;
                constexpr bool DO_RD = decltype(rd_c)::value && !(ABL & 2);
                constexpr bool DO_DMA = decltype(dma_c)::value && !(ABL & 1);
                const int64_t aoff = DO_DMA ? a_koff(s) : 0;
                const Bases bs = DO_DMA ? bases_of(dbuf) : Bases{};
                // (HN: NJ channel blocks; the W reads / pieces move from J = 4 / 2 to 2 / 3 (1 / 1
                // for NJ = 2), I < NJ)
                constexpr int JW = HN ? (NJ > 2 ? 2 : 1) : 4;
                static_for<8>([&](auto i_c) __attribute__((always_inline)) {
                    constexpr int I = decltype(i_c)::value;
                    constexpr bool WI = !HN || I < NJ;  // a W block to read / a W piece to issue
                    static_for<NJ>([&](auto j_c) __attribute__((always_inline)) {
                        constexpr int J = decltype(j_c)::value;
                        if constexpr (KIND == 0) {
                            if constexpr (DO_RD && J == 0)
                                fa[1 - H][I] = *(const u32x4*)(rbuf + a_base + I * 2048 + fo1);
                            if constexpr (DO_RD && J == JW && WI)
                                fw[1][I] = *(const u32x4*)(rbuf + w_base + I * 2048 + fo1);
                            amma<CT, 4 * (8 * I + J), ZERO>(fw[0][J], fa[H][I]);
                        } else if constexpr (KIND == 1) {
                            if constexpr (DO_RD && J == 0 && I > 0)
                                fa[1 - H][I - 1] = *(const u32x4*)(rbuf + a_base + (I - 1) * 2048 + fo0);
                            if constexpr (DO_DMA && J == JW) dma_piece(dbuf, i_c, s, aoff, bs);
                            if constexpr (RQ >= 0 && !HN && (J == 2 || J == 6))
                                xres_piece(rqbuf, i_c, std::integral_constant<int, J / 4>{}, RQ, 0);
                            amma<CT, 4 * (8 * I + J), false>(fw[0][J], fa[1 - H][I]);
                        } else {
                            if constexpr (DO_RD && J == 0 && I == 0)
                                fa[1 - H][7] = *(const u32x4*)(rbuf + a_base + 7 * 2048 + fo0);
                            if constexpr (DO_RD && J == JW && WI)
                                fw[0][I] = *(const u32x4*)(rbuf + w_base + I * 2048 + fo0);
                            if constexpr (DO_DMA && J == (HN ? NJ - 1 : 2) && WI)
                                dma_piece(dbuf, std::integral_constant<int, 8 + I>{}, s, aoff, bs);
                            if constexpr (RQ >= 0 && !HN && (J == 2 || J == 6))
                                xres_piece(rqbuf, i_c, std::integral_constant<int, J / 4>{}, RQ, 0);
                            amma<CT, 4 * (8 * I + J), false>(fw[1][J], fa[H][I]);
                        }
                        __builtin_amdgcn_sched_barrier(0);
                    });
                });
                if constexpr (KIND == 2 && DO_RD) __builtin_amdgcn_s_waitcnt(kLgkm0);
            };
            using K0 = std::integral_constant<int, 0>;
            using K1 = std::integral_constant<int, 1>;
            using K2 = std::integral_constant<int, 2>;
            // K-tile t in buffer `b` (the next one in `o`), A_hi in fa[H]
            // vm: the mid wait (K-tile 0 of a walked tile: 63 = none on vmcnt -- K-tile 1 was issued
            // before the previous epilogue's residual loads, which that epilogue waited for, and
            // vmcnt retires in issue order -- so that epilogue's last stores stay in flight)
            // rql: the last K-tile of a residual-through-LDS unit -- quarter (0, 0) into `o` (K-tile
            // nk - 2's buffer) in phase B1, quarter (0, 1) into `b` in B2, 2 pieces per row block
            // (both buffers are free past this K-tile's mid barrier)
            auto x3_ktile_q = [&](auto h_c, auto zero_c, auto rd_c, auto dma_c, auto rql_c, int t, char* b, char* o,
                                  int vm) __attribute__((always_inline)) {
                constexpr bool rql = decltype(rql_c)::value;
                x3_phase(h_c, K0{}, zero_c, T_{}, F_{}, b, nullptr, 0, std::integral_constant<int, -1>{}, nullptr);
                if (vm == 63)
                    __builtin_amdgcn_s_waitcnt(kLgkm0);
                else if (vm == 32)
                    __builtin_amdgcn_s_waitcnt(kVm32Lgkm0);
                else
                    __builtin_amdgcn_s_waitcnt(kVm0Lgkm0);
                pinned_barrier();
                x3_phase(h_c, K1{}, F_{}, rd_c, dma_c, o, b, t + 2, std::integral_constant<int, rql ? 0 : -1>{}, o);
                x3_phase(h_c, K2{}, F_{}, rd_c, dma_c, o, b, t + 2, std::integral_constant<int, rql ? 1 : -1>{}, b);
            };
            auto x3_ktile = [&](auto h_c, auto zero_c, auto rd_c, auto dma_c, int t, char* b, char* o, int vm = 0)
                                __attribute__((always_inline)) {
                x3_ktile_q(h_c, zero_c, rd_c, dma_c, std::false_type{}, t, b, o, vm);
            };
            // a walked tile after a residual-through-LDS epilogue: K-tile 1 landed, that
            // epilogue's 32 H1 stores may stay in flight (32); after a global-residual one nothing
            // on vmcnt (63); the first tile drains
            const int vm0 = first ? 0 : (x3_prev_xres ? 32 : 63);
            if (nk > 2)
                x3_ktile(C0{}, T_{}, T_{}, T_{}, 0, buf0, buf1, vm0);
            else if (nk == 2)
                x3_ktile(C0{}, T_{}, T_{}, F_{}, 0, buf0, buf1, vm0);
            else
                x3_ktile(C0{}, T_{}, F_{}, F_{}, 0, buf0, buf1, vm0);
            int t = 1;
            for (; t + 3 < nk; t += 2) {
                x3_ktile(C1{}, F_{}, T_{}, T_{}, t, buf1, buf0);
                x3_ktile(C0{}, F_{}, T_{}, T_{}, t + 1, buf0, buf1);
            }
            if (t + 2 < nk) {
                x3_ktile(C1{}, F_{}, T_{}, T_{}, t, buf1, buf0);
                x3_ktile(C0{}, F_{}, T_{}, F_{}, t + 1, buf0, buf1);
                if (xres) {
                    xres_prep();
                    x3_ktile_q(C1{}, F_{}, F_{}, F_{}, std::true_type{}, t + 2, buf1, buf0, 0);
                } else {
                    x3_ktile(C1{}, F_{}, F_{}, F_{}, t + 2, buf1, buf0);
                }
            } else if (t + 1 < nk) {
                x3_ktile(C1{}, F_{}, T_{}, F_{}, t, buf1, buf0);
                if (xres) {
                    xres_prep();
                    x3_ktile_q(C0{}, F_{}, F_{}, F_{}, std::true_type{}, t + 1, buf0, buf1, 0);
                } else {
                    x3_ktile(C0{}, F_{}, F_{}, F_{}, t + 1, buf0, buf1);
                }
            } else if (t < nk) {
                x3_ktile(C1{}, F_{}, F_{}, F_{}, t, buf1, buf0);
            }
            asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
            // tile walk (the 1x1 + residual layers): every wave has passed the last K-tile's
            // barrier after its last LDS reads, so both buffers take the next tile's K-tiles 0
            // and 1 now, ahead of this tile's epilogue loads and stores (in flight under the
            // next tile's first K-tiles); em0 / en0 keep this tile's origin
            const int em0 = m0, en0 = n0;
            const int erole = role, esidx = sidx, esq = sq;
            // residual through LDS: quarters (0, *) sit in the buffers of K-tiles nk - 2 / nk - 1
            char* const qb0 = (nk & 1) ? buf1 : buf0;  // quarter (*, 0): K-tile nk - 2's buffer
            char* const qb1 = (nk & 1) ? buf0 : buf1;
            // the half's residual rows from LDS into rr (accumulator layout as the global loads)
            auto xres_read = [&](u32x4 (&rr)[8][2][2]) __attribute__((always_inline)) {
                int ln = lane, wv = widu;
                asm volatile("" : "+v"(ln));
                launder_s(wv);
                const char* qb = (wv & 1) ? qb1 : qb0;  // wave column wc = wid & 1
                const int swz = (((ln >> 3) & 1) * 4 + ((ln & 7) >> 1)) & 7;
                const int g = ln >> 4;
                const int cc = (g & 1) * 2 + (g >> 1);  // c0 / 8
                const char* rowp = qb + (2 * ((wv >> 1) * 16 + ((ln >> 3) & 1))) * 1024 + (ln & 7) * 128;
#pragma unroll
                for (int i = 0; i < 8; ++i)
#pragma unroll
                    for (int jp = 0; jp < 2; ++jp)
#pragma unroll
                        for (int hl = 0; hl < 2; ++hl)
                            rr[i][jp][hl] = *(const u32x4*)(rowp + (4 * i + jp) * 1024 + (((hl * 4 + cc) ^ swz) << 4));
            };
            constexpr int OB = X3 == 2 ? 4 : 2;  // output element bytes
            typedef float f32x2 __attribute__((ext_vector_type(2)));
            typedef int i32x2 __attribute__((ext_vector_type(2)));
            const bool has_r = p.R != nullptr;
            // the epilogue's lane values from a fresh laundered copy (those of the tile top would
            // otherwise stay live across the K loop, which has no VGPRs to spare)
            int eln = lane, ewv = widu;
            asm volatile("" : "+v"(eln));
            launder_s(ewv);
            const int egrp = eln >> 4, er16 = eln & 15;
            const int ec0 = 8 * ((egrp & 1) * 2 + (egrp >> 1));
            const int ewr = ewv >> 1, ewc = ewv & 1;
            // split epilogue of channel half HH (64 channels per wave) with the residual rows in rr
            // (WITH_R) -- the arithmetic of gemm::epilogue_tp_x3, so the same bits: BN as
            // v_pk_mul_f32 + v_pk_add_f32, ReLU as an integer max on the f32 bits,
            // v_permlane16_swap to 8 consecutive channels per lane, residual hi + lo added in f32,
            // output split into hi / lo halves (16 bytes each) or f32 rows (X3 = 2)
            auto x3_half = [&](auto hh_c, auto wr_c, const u32x4 (&rr)[8][2][2], __amdgpu_buffer_rsrc_t y_rsrc)
                               __attribute__((always_inline)) {
                constexpr int HH = decltype(hh_c)::value;
                constexpr bool WITH_R = decltype(wr_c)::value && !(ABL & 8);
                const int nw = en0 + ewc * (TN / 2) + 64 * HH;
                f32x2 sc[4][2], sh[4][2];
#pragma unroll
                for (int j = 0; j < NB; ++j) {
                    const int n = nw + 16 * j + 4 * egrp;
                    const f32x4 s4 = *(const f32x4*)&s_scale[n];
                    const f32x4 h4 = *(const f32x4*)&s_shift[n];
                    sc[j][0] = f32x2{s4[0], s4[1]};
                    sc[j][1] = f32x2{s4[2], s4[3]};
                    sh[j][0] = f32x2{h4[0], h4[1]};
                    sh[j][1] = f32x2{h4[2], h4[3]};
                }
                static_for<8>([&](auto i_c) __attribute__((always_inline)) {
                    constexpr int I = decltype(i_c)::value;
                    const int m = em0 + ewr * 128 + 16 * I + er16;
                    float v4[4][4];  // [block j][element]: BN + ReLU, accumulator layout
                    static_for<NB>([&](auto j_c) __attribute__((always_inline)) {
                        constexpr int J = decltype(j_c)::value;
                        constexpr int R = 4 * (8 * I + 4 * HH + J);
                        f32x2 v[2] = {f32x2{aread<R>(), aread<R + 1>()}, f32x2{aread<R + 2>(), aread<R + 3>()}};
                        if (erole == kOwner) owner_add(std::integral_constant<int, R>{}, esidx, v);
#pragma unroll
                        for (int q = 0; q < 2; ++q) {
                            f32x2 x = v[q] * sc[J][q];
                            x = x + sh[J][q];
                            if (p.relu) {
                                i32x2 xi = __builtin_bit_cast(i32x2, x);
                                xi = __builtin_elementwise_max(xi, i32x2{0, 0});
                                x = __builtin_bit_cast(f32x2, xi);
                            }
                            v4[J][2 * q] = x[0];
                            v4[J][2 * q + 1] = x[1];
                        }
                    });
#pragma unroll
                    for (int jp = 0; jp < NB / 2; ++jp) {
                        float* x = v4[2 * jp];
                        float* y = v4[2 * jp + 1];
                        asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\tv_permlane16_swap_b32 %2, %3\n\t"
                                     "v_permlane16_swap_b32 %4, %5\n\tv_permlane16_swap_b32 %6, %7"
                                     : "+v"(x[0]), "+v"(y[0]), "+v"(x[1]), "+v"(y[1]), "+v"(x[2]), "+v"(y[2]),
                                       "+v"(x[3]), "+v"(y[3]));
                        float v[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
                        if constexpr (WITH_R) {
                            // v + (rh + rl): the exact pair sums as mixed FMAs, then one f32 add each
                            const u32x4 rh = rr[I][jp][0], rl = rr[I][jp][1];
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                float t0, t1;
                                gemm::x3_res_sum2(rh[e], rl[e], t0, t1);
                                v[2 * e] += t0;
                                v[2 * e + 1] += t1;
                            }
                        }
                        const bool in = m < p.M;
                        if constexpr (X3 == 2) {
                            const uint32_t yo =
                                in ? (uint32_t)(((size_t)(m - em0) * p.ldy + nw + 32 * jp + ec0) * 4) : 0xFFFFFFE0u;
                            __builtin_amdgcn_raw_buffer_store_b128(
                                __builtin_bit_cast(u32x4, f32x4{v[0], v[1], v[2], v[3]}), y_rsrc, yo, 0, 0);
                            __builtin_amdgcn_raw_buffer_store_b128(
                                __builtin_bit_cast(u32x4, f32x4{v[4], v[5], v[6], v[7]}), y_rsrc, yo + 16, 0, 0);
                        } else {
                            // hi = f16(v), lo = f16(v - hi) (v_fma_mixlo/mixhi: one rounding, as before)
                            u32x4 oh, ol;
                            float t = 0.f;
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                oh[e] = gemm::x3_hi2(v[2 * e], v[2 * e + 1]);
                                ol[e] = gemm::x3_split_lo2(oh[e], v[2 * e], v[2 * e + 1]);
                                t = gemm::x3_absmax2(t, v[2 * e], v[2 * e + 1]);
                            }
                            // (per 8 values: a running max over the half costs a VGPR the K
                            // loop does not have)
                            gemm::x3_range_flag(in ? t : 0.f, p.scale, p.N);
                            const uint32_t yo =
                                in ? (uint32_t)(((size_t)(m - em0) * p.ldy + 2 * nw + 64 * jp + ec0) * 2) : 0xFFFFFF00u;
                            if constexpr ((ABL & 16) != 0) {  // (measurement builds: no output stores)
                                asm volatile("" ::"v"(oh), "v"(ol));
                            } else {
                                __builtin_amdgcn_raw_buffer_store_b128(oh, y_rsrc, yo, 0, 0);
                                __builtin_amdgcn_raw_buffer_store_b128(ol, y_rsrc, yo + 64, 0, 0);
                            }
                        }
                    }
                });
            };
            auto y_rsrc_of = [&]() __attribute__((always_inline)) {
                // the output resource starts at the tile's first row (outputs past 2^31 bytes)
                const size_t y_rest = (size_t)(p.M - em0) * p.ldy * OB;
                return make_rsrc((const char*)p.Y + (size_t)em0 * p.ldy * OB,
                                 clamp_range31(y_rest));
            };
            if (xres) {
                // ---- residual through LDS: half 0 from quarters (0, *) into registers, quarters
                // (1, *) into the same buffers (landing under half 0's epilogue), half 1, then the
                // next tile's K-tiles 0 and 1 (in flight under half 1's epilogue) ----
                u32x4 rr[8][2][2];
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's quarter (0, *) pieces
                pinned_barrier();
                xres_read(rr);
                __builtin_amdgcn_s_waitcnt(kLgkm0);
                pinned_barrier();  // every wave has its half-0 rows: the buffers take quarters (1, *)
                static_for<8>([&](auto i_c) __attribute__((always_inline)) {
                    xres_piece(qb0, i_c, std::integral_constant<int, 0>{}, 0, 1);
                    xres_piece(qb0, i_c, std::integral_constant<int, 1>{}, 0, 1);
                    xres_piece(qb1, i_c, std::integral_constant<int, 0>{}, 1, 1);
                    xres_piece(qb1, i_c, std::integral_constant<int, 1>{}, 1, 1);
                });
                if (erole == kOwner) owner_wait(esidx);
                const __amdgpu_buffer_rsrc_t y_rsrc = y_rsrc_of();
                x3_half(std::integral_constant<int, 0>{}, T_{}, rr, y_rsrc);
                // quarters (1, *) landed (younger: the 32 H0 stores)
                asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
                pinned_barrier();
                xres_read(rr);
                __builtin_amdgcn_s_waitcnt(kLgkm0);
                pinned_barrier();
                // the next tile's K-tiles 0 and 1 ahead of the H1 stores: its first waits leave
                // those in flight (vmcnt retires in issue order)
                if (has_next) {
                    setup(next);
                    stage_01();
                }
                x3_half(std::integral_constant<int, 1>{}, T_{}, rr, y_rsrc);
                if (erole == kOwner) owner_done(esidx);
            } else {
                // tile walk (the 1x1 + residual layers without the LDS form, VP3D_A4_WALK=2): every
                // wave has passed the last K-tile's barrier after its last LDS reads, so both
                // buffers take the next tile's K-tiles 0 and 1 now, ahead of this tile's epilogue
                // loads and stores (in flight under the next tile's first K-tiles)
                if (has_next) {
                    setup(next);
                    stage_01();
                }
                if (erole == kHelper) {
                    helper_store(esidx, esq);
                    x3_prev_res = false;
                    x3_prev_xres = false;
                    if (!has_next) break;
                    tix = next;
                    first = false;
                    continue;
                }
                if (erole == kOwner) owner_wait(esidx);
                const __amdgpu_buffer_rsrc_t y_rsrc = y_rsrc_of();
                const int rrow0 = has_r ? res_row(p, em0) : 0;
                const __amdgpu_buffer_rsrc_t rx_rsrc =
                    make_rsrc(has_r ? (const f16*)p.R + (int64_t)rrow0 * p.ldr : (const f16*)p.A, 0x7FFFFFFFu);
                // the residual of a whole half (8 row blocks x 2 x hi / lo, 128 VGPRs) loaded up
                // front -- epilogue_tp_x3 loads it one row block ahead, a latency per row block
                auto global_half = [&](auto hh_c) __attribute__((always_inline)) {
                    constexpr int HH = decltype(hh_c)::value;
                    const int nw = en0 + ewc * (TN / 2) + 64 * HH;
                    u32x4 rr[8][2][2];
                    if (has_r && !(ABL & 8)) {
#pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            int m = em0 + ewr * 128 + 16 * i + er16;
                            m = m < p.M ? m : p.M - 1;  // valid address; rows past M are never stored
                            const int off = ((res_row(p, m) - rrow0) * p.ldr + 2 * nw + ec0) * 2;
#pragma unroll
                            for (int jp = 0; jp < NB / 2; ++jp) {  // (quarter-N: the wave's 32 channels only)
                                rr[i][jp][0] = __builtin_bit_cast(
                                    u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx_rsrc, off + 128 * jp, 0, 0));
                                rr[i][jp][1] = __builtin_bit_cast(
                                    u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx_rsrc, off + 128 * jp + 64, 0, 0));
                            }
                        }
                        x3_half(hh_c, T_{}, rr, y_rsrc);
                    } else {
                        x3_half(hh_c, F_{}, rr, y_rsrc);
                    }
                };
                if constexpr ((ABL & 32) == 0) {  // (measurement builds: ABL bit 5 skips the epilogue)
                    global_half(std::integral_constant<int, 0>{});
                    if constexpr (!HN) global_half(std::integral_constant<int, 1>{});
                }
                if (erole == kOwner) owner_done(esidx);
            }
            x3_prev_res = has_r;
            x3_prev_xres = xres;
            if (!has_next) break;
            tix = next;
            first = false;
            continue;
        } else {
        // K-tile 0 (phase A initialises the accumulators: C = 0), then the steady state (both
        // follow-up K-tiles exist: no branch inside a K-tile), then the last two K-tiles (with
        // nk >= 3 always the tail's last two calls)
        // mid(0) of a later tile: K-tile 1 landed, younger stores may stay in flight (32; with
        // a residual the H1 stores only, 16)
        const int vm0 = first ? 0 : prev_lres ? 16 : 32;
        if (nk > 2)
            ktile(T_{}, T_{}, T_{}, 0, buf0, buf1, -1, vm0);
        else if (nk == 2)
            ktile(T_{}, T_{}, F_{}, 0, buf0, buf1, -1, vm0);
        else
            ktile(T_{}, F_{}, F_{}, 0, buf0, buf1, -1, vm0);
#ifdef VP3D_ABLATION
        if (first) stamp(1);
#endif
        const int em0 = m0, en0 = n0;
        enk = nk;
        const int erole = role, esidx = sidx, esq = sq;
        const bool elres = lres;
        // the next tile's addressing once this tile's last operand DMA has been issued
        auto next_setup = [&]() __attribute__((always_inline)) {
            if (has_next) setup(next);
        };
        // without a residual: the next tile's K-tiles 0 and 1 in phase B of the last K-tile
        // (both buffers free), two pieces per DMA slot
        auto last_ktile = [&](int t, char* b, char* o) __attribute__((always_inline)) {
            phase(C0{}, F_{}, T_{}, F_{}, b, fo1, nullptr, 0, -1);
            mid(lres ? 16 : 0);
            if (lres || !has_next) {
                phase(C1{}, F_{}, F_{}, F_{}, o, fo0, b, 0, res1);
            } else {
                next_setup();
                phase(C1{}, F_{}, F_{}, F_{}, o, fo0, b, 0, -1);
                stage_01();
            }
        };
        int t = 1;
        for (; t + 3 < nk; t += 2) {
            ktile(F_{}, T_{}, T_{}, t, buf1, buf0, -1, 0);
            ktile(F_{}, T_{}, T_{}, t + 1, buf0, buf1, -1, 0);
        }
        // 0..3 K-tiles left, t odd (buffer 1)
        if (t + 2 < nk) {  // three: t, t + 1, t + 2
            ktile(F_{}, T_{}, T_{}, t, buf1, buf0, -1, 0);
            ktile(F_{}, T_{}, F_{}, t + 1, buf0, buf1, res0, 0);
            last_ktile(t + 2, buf1, buf0);
        } else if (t + 1 < nk) {  // two
            ktile(F_{}, T_{}, F_{}, t, buf1, buf0, res0, 0);
            last_ktile(t + 1, buf0, buf1);
        } else if (t < nk) {  // one (nk <= 2: no residual parts)
            last_ktile(t, buf1, buf0);
        }
        // the last MFMAs' results -> v_accvgpr_read (inline-asm MFMAs are not tracked by the
        // compiler's hazard recognizer)
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#ifdef VP3D_ABLATION
        stamp(2);
        if (trc && tid == 0) trc[9] = mid_cyc;
#endif

        if (erole == kHelper) {  // split-K helper: no epilogue (never followed by another unit)
            helper_store(esidx, esq);
            break;
        }
        if (erole == kOwner) owner_wait(esidx);
        const int own_si = erole == kOwner ? esidx : -1;
        // the output resource starts at the tile's first row (outputs past 2^31 bytes: the
        // store offsets stay 32-bit and tile-relative; rows past M fall outside the range)
        const size_t y_rest = (size_t)(p.M - em0) * p.ldy * sizeof(CT);
        const __amdgpu_buffer_rsrc_t y_rsrc =
            make_rsrc((const CT*)p.Y + (size_t)em0 * p.ldy, clamp_range31(y_rest));
        if (!HN && elres) {
            // residual part h into registers once landed (every wave's pieces: after the
            // barrier), then its buffer takes the next tile's K-tile h (nk even: part h sits in
            // buffer h) before the half-h stores: issue order part 0, part 1, K-tile 0, H0
            // stores, K-tile 1, H1 stores -- the next tile's first waits pass the stores
            auto part = [&](auto h_c) __attribute__((always_inline)) {
                constexpr int H = decltype(h_c)::value;
                // younger than part h: part 1 (H = 0), or K-tile 0 and the H0 stores (H = 1)
                if (H == 0 || !has_next)
                    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                else
                    asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
                pinned_barrier();
#pragma unroll
                for (int i = 0; i < 8; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) resr[i][j] = *res_addr(H, i, j);
                if (has_next) {
                    __builtin_amdgcn_s_waitcnt(kLgkm0);
                    pinned_barrier();
                    if (H == 0) next_setup();
                    const int64_t o = a_koff(H);
                    const Bases bh = bases_of(H == 0 ? buf0 : buf1);
                    static_for<16>([&](auto i_c) __attribute__((always_inline)) {
                        dma_piece(H == 0 ? buf0 : buf1, i_c, H, o, bh);
                    });
                }
                epi_fast(h_c, true, em0, en0, y_rsrc, own_si);
            };
            part(H0{});
            part(H1{});
        } else {  // no residual (the eligibility check leaves no residual with nk < 3)
            epi_fast(H0{}, false, em0, en0, y_rsrc, own_si);
            if constexpr (!HN) epi_fast(H1{}, false, em0, en0, y_rsrc, own_si);
        }
        if (erole == kOwner) owner_done(esidx);
        prev_lres = elres;
        if (!has_next) break;
        tix = next;
        first = false;
        }  // X3 == 0
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
    if (p.R && p.Kp / GK < 3) return false;  // the residual lands in LDS during the last two K-tiles
    if (p.Ktap % GK != 0 || p.Kp % GK != 0 || p.lda % 8 != 0) return false;
    if (p.N % GN != 0 || p.N > GMAXN || p.ldy % 8 != 0 || (p.R && p.ldr % 8 != 0)) return false;
    if ((reinterpret_cast<uintptr_t>(p.A) & 15) || (reinterpret_cast<uintptr_t>(p.Y) & 15) ||
        (p.R && (reinterpret_cast<uintptr_t>(p.R) & 15)))
        return false;
    return (size_t)p.N * p.Kp < (1u << 31);
}

static int a4_hn_tail(const ConvGemmParams& p, int ntiles, bool x3, int* level = nullptr);
static bool a4_tail_split(const ConvGemmParams& p, int mt_tail, int level, bool need_ws);

bool conv_gemm_a4_x3_eligible(const ConvGemmParams& p, bool out_f32) {
    if (p.Ktap % GK != 0 || p.Kp % GK != 0 || p.lda % 8 != 0) return false;
    if (p.N % GN != 0 || p.N > GMAXN || p.ldy % (out_f32 ? 4 : 8) != 0 || (p.R && p.ldr % 8 != 0)) return false;
    if ((reinterpret_cast<uintptr_t>(p.A) & 15) || (reinterpret_cast<uintptr_t>(p.Y) & 15) ||
        (reinterpret_cast<uintptr_t>(p.W) & 15) || (p.R && (reinterpret_cast<uintptr_t>(p.R) & 15)))
        return false;
    // enough tiles to fill the CUs (as the 16-bit dispatch: >= 384 tiles of 256 x 256), or a
    // half-N or split plan that does
    const int ntiles = ((p.M + GM - 1) / GM) * (p.N / GN);
    if (!conv_gemm_a4_fills(p) && a4_hn_tail(p, ntiles, true) == 0) return false;
    return (size_t)p.N * p.Kp < (1u << 31);
}

static int a4_cus() {
    static const int ncu = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 0;
        return n & ~7;
    }();
    return ncu;
}

// Split-K plan of a launch's partial last round: L = the tiles past the last whole round of the
// chip's CUs, each split into S = CUs / L units (<= 4) of an equal whole number (even, >= 4) of
// K-tiles, so the last round is S x L <= CUs units of 1 / S the work.  Config 4 at N = 8 (8,192
// windows per GPU) leaves L = 128 in every block (block 4 has 128 tiles in all) -> S = 2.  Taken
// only for long K (>= 64 K-tiles: the split-fp16 k3 convs) over few rounds (< 8): the helper's
// 256 KiB of partial sums, the owner's wait and adds and the split variant's extra scalar
// registers (spilled to VGPR lanes) cost about an epilogue, and every unit of the launch runs
// the split variant.  Measured at B = 8,192 (profiles/r04q_split_k_ab.txt): f16x3 block-2 /
// 3 / 4 k3 0.977 / 0.361 / 0.154 vs 0.994 / 0.387 / 0.187 ms whole-tile; block-1 k3 (13.5
// rounds) 2.707 vs 2.692; every 1x1 (16-32 K-tiles) and every bf16 layer slower (bf16 block-3
// 1x1 0.100 vs 0.061 ms).  Needs the handle's workspace (sk_part); VP3D_A4_SPLIT=0
// (measurement; read at every launch) turns it off, 2 takes it wherever it fits.  Returns the
// plan in q.sk_* (sk_split 0: none).
static void a4_split_plan(ConvGemmParams& q, int ntiles, int nk, bool need_ws = true) {
    q.sk_split = q.sk_full = q.sk_left = 0;
    const char* e = getenv("VP3D_A4_SPLIT");
    const int mode = e ? atoi(e) : 1;
    if (mode == 0 || (need_ws && (!q.sk_part || !q.sk_flag))) return;
    const int ncu = a4_cus();
    if (ncu <= 0 || ncu > 256) return;  // the workspace holds one round of 256 slots
    if (mode == 1 && (nk < 64 || ntiles >= 8 * ncu)) return;
    const int L = ntiles % ncu;
    if (L == 0) return;
    int S = ncu / L;
    S = S > 4 ? 4 : S;
    while (S >= 2 && (nk % S != 0 || nk / S < 4 || (nk / S) % 2 != 0)) --S;
    if (S < 2) return;
    q.sk_full = ntiles - L;
    q.sk_split = S;
    q.sk_left = L;
}

// the tile count from which a4 is the kernel of a 16-bit layer (fewer: q64 / the 128 x 128
// kernel), unless a split plan fills the chip (config 4's block 4 at N = 8: 128 tiles)
// Half-N plan of a launch's partial last round (round 5): with L <= CUs / 2 tiles past the last
// whole round, their L / 4 M-tiles (N = 1024) run as 2L units of 256 x 128 in a second launch
// (conv_gemm_a4<..., HN>) after the whole rounds -- every output in the whole tile's K order,
// so bit-identical across batch sizes (split-K sums a tile's K in S chains).  Layers without a
// residual, and the f16x3 1x1 + residual layers (half tiles load their residual half globally;
// the whole rounds before them are walked as usual).  Measured same box
// (profiles/r05_a4_half_n_tail_ab.txt): f16x3 at 8,192 windows every conv faster than split-K /
// whole tiles (block-4 k3 0.122 vs 0.151 ms, 1x1 0.056 vs 0.079), step +2.4 % (0.946 of 65,536);
// 16-bit operands only where the layer has no whole round (block 4 at 8,192: 0.060 vs 0.085
// ms; 1,024 windows +8 %) -- after whole rounds their half tiles, DMA-issue-bound at 12 pieces
// per 64 MFMAs, ran no faster than the whole-tile round (block 3 at 8,192: 0.157 vs 0.148).
// f16x3 tails of <= a quarter round run as 4L quarter-N tiles of 256 x 64 (level 2): sequence
// mode's 4-tile tails and config 4 at 1,024 windows (blocks 3, 4), +1 % / +3.4 % same box
// (profiles/r05_a4_quarter_n_tail_ab.txt).  VP3D_A4_HN=0 (measurement) turns it off, 1 keeps
// half tiles only; VP3D_A4_SPLIT=2 (the split-K test) takes precedence.  Returns the M-tiles
// of the tail (0: none) and in *level 1 (half-N) or 2 (quarter-N).
static int a4_hn_tail(const ConvGemmParams& p, int ntiles, bool x3, int* level) {
    const char* e = getenv("VP3D_A4_HN");
    if (e && e[0] == '0') return 0;
    const char* sp = getenv("VP3D_A4_SPLIT");
    if (sp && atoi(sp) == 2) return 0;
    const int ncu = a4_cus();
    const int ntn = p.N / GN;
    // (the f16x3 1x1 + residual layers too: their half tiles load the residual half globally)
    if ((p.R != nullptr && !x3) || ncu <= 0 || ntn <= 0) return 0;
    const int L = ntiles % ncu;
    if (L == 0 || 2 * L > ncu || L % ntn != 0 || (!x3 && ntiles >= ncu)) return 0;
    // f16x3 tails of <= a quarter round: 4L quarter-N units of 256 x 64 (VP3D_A4_HN=1: half only)
    if (level) *level = x3 && 4 * L <= ncu && !(e && e[0] == '1') ? 2 : 1;
    return L / ntn;
}

// Split-K tail (conv_gemm_tail.hip, round 6): an f16x3 tail of <= a quarter round (the quarter-N
// level) after at least one whole round -- sequence mode's 4-tile tails -- runs as (N / 64) x S
// slices of its K range over every CU plus a reduction launch, instead of 4L quarter-N tiles each
// a full-K chain on one CU.  Not the whole tiles' bits (S partial chains), so the half-N tails
// of config 4's shards (8 x 8,192 windows == one 65,536 forward, bit for bit) keep their tiles.
// The 16-bit layers (bf16 / fp16), which run such tails as a fifth round of whole tiles, take the
// same split tail (launch_conv_gemm_tail16).  VP3D_A4_TAIL=hn (measurement, read at every launch)
// keeps the quarter-N tiles / whole tiles; VP3D_A4_SPLIT=0 as well.
static bool a4_tail_split(const ConvGemmParams& p, int mt_tail, int level, bool need_ws) {
    if (level != 2 || mt_tail <= 0) return false;
    const char* e = getenv("VP3D_A4_TAIL");
    if (e && strcmp(e, "hn") == 0) return false;
    const char* sp = getenv("VP3D_A4_SPLIT");  // 0: whole tiles only (no split-K of any kind)
    if (sp && atoi(sp) == 0) return false;
    const int mt0 = (p.M + GM - 1) / GM - mt_tail;
    if (mt0 <= 0) return false;  // no whole round: the quarter-N tiles (bit-identical across batch sizes)
    return conv_gemm_tail_fits(p, mt0 * GM, a4_cus(), need_ws);
}

bool conv_gemm_a4_would_split(const ConvGemmParams& p) {
    const int ntiles = ((p.M + GM - 1) / GM) * (p.N / GN);
    int level = 1;
    const int hn = a4_hn_tail(p, ntiles, true, &level);
    if (hn > 0) return a4_tail_split(p, hn, level, false);  // (the split workspace: f16x3 layers)
    ConvGemmParams q = p;
    a4_split_plan(q, ntiles, p.Kp / GK, false);
    return q.sk_split > 1;
}

bool conv_gemm_a4_fills(const ConvGemmParams& p) {
    const int ntiles = ((p.M + GM - 1) / GM) * (p.N / GN);
    if (ntiles >= 384) return true;
    if (a4_hn_tail(p, ntiles, false) > 0) return true;  // the 16-bit dispatch: the layer as 2L half tiles
    ConvGemmParams q = p;
    a4_split_plan(q, ntiles, p.Kp / GK);
    return q.sk_split > 1;
}

template <typename CT, int X3>
static void a4_launch(const ConvGemmParams& p, dim3 grid, bool split, hipStream_t stream) {
    if (split)
        hipLaunchKernelGGL((conv_gemm_a4<CT, 0, X3, true, true>), grid, dim3(256), 0, stream, p);
    else
        hipLaunchKernelGGL((conv_gemm_a4<CT, 0, X3, true, false>), grid, dim3(256), 0, stream, p);
}

// the whole rounds (M-tiles below ntm - mt_tail, if any; walked by one workgroup per CU when
// `walk_cus` > 0) then the tail as half-N units
template <typename CT, int X3>
static void a4_launch_whole(const ConvGemmParams& p, int mt0, hipStream_t stream, int walk_cus) {
    if (mt0 > 0) {
        ConvGemmParams q = p;
        q.M = mt0 * GM;
        q.sk_split = q.sk_full = q.sk_left = 0;
        const int tiles = mt0 * (p.N / GN);
        const dim3 g(walk_cus > 0 && tiles > walk_cus ? walk_cus : tiles);
        hipLaunchKernelGGL((conv_gemm_a4<CT, 0, X3, true, false>), g, dim3(256), 0, stream, q);
    }
}

template <typename CT, int X3>
static void a4_launch_hn(const ConvGemmParams& p, int mt_tail, hipStream_t stream, int walk_cus = 0, int level = 1) {
    const int ntm = (p.M + GM - 1) / GM;
    const int mt0 = ntm - mt_tail;
    a4_launch_whole<CT, X3>(p, mt0, stream, walk_cus);
    ConvGemmParams t = p;
    t.sk_split = t.sk_left = 0;
    t.sk_full = mt0;  // the HN launch's first M-tile
    if constexpr (X3 != 0) {
        if (level == 2) {
            hipLaunchKernelGGL((conv_gemm_a4<CT, 0, X3, true, false, 2>), dim3(mt_tail * (p.N / (GN / 4))), dim3(256),
                               0, stream, t);
            return;
        }
    }
    hipLaunchKernelGGL((conv_gemm_a4<CT, 0, X3, true, false, 1>), dim3(mt_tail * (p.N / (GN / 2))), dim3(256), 0,
                       stream, t);
}

#ifdef VP3D_ABLATION
// measurement builds (tools/ubench/x3_1x1_check): VP3D_ABL bits 1 no loop DMA, 2 no loop
// fragment reads, 8 no residual loads, 16 no output stores, 32 no epilogue (timing only)
template <int ABL>
static void a4_x3_abl(const ConvGemmParams& p, dim3 grid) {
    hipLaunchKernelGGL((conv_gemm_a4<_Float16, ABL, 1, true, false>), grid, dim3(256), 0, 0, p);
}
#endif

hipError_t launch_conv_gemm_a4_x3(const ConvGemmParams& p_in, bool out_f32, hipStream_t stream) {
    // the 1x1 + residual layers walk their tiles (one workgroup per CU, as launch_conv_gemm_a4);
    // VP3D_A4_WALK 0: never, 2: every layer
    const int ntiles = ((p_in.M + GM - 1) / GM) * (p_in.N / GN);
    ConvGemmParams p = p_in;
    const char* we = getenv("VP3D_A4_WALK");
    const int walk_mode = we ? atoi(we) : 1;
    int hn_level = 1;
    const int hn_tail = walk_mode == 2 ? 0 : a4_hn_tail(p, ntiles, true, &hn_level);
#ifndef VP3D_ABLATION
    if (hn_tail > 0) {
        // the whole rounds walked as without the tail (the 1x1 + residual layers)
        const int wc = walk_mode > 0 && p.R != nullptr ? a4_cus() : 0;
        if (a4_tail_split(p, hn_tail, hn_level, true)) {
            // a tail of <= a quarter round after whole rounds (sequence mode): split over every
            // CU in its K range too (conv_gemm_tail.hip), not as 4L quarter-N full-K chains
            const int mt0 = (p.M + GM - 1) / GM - hn_tail;
            if (out_f32)
                a4_launch_whole<_Float16, 2>(p, mt0, stream, wc);
            else
                a4_launch_whole<_Float16, 1>(p, mt0, stream, wc);
            return launch_conv_gemm_tail_x3(p, mt0 * GM, out_f32, a4_cus(), stream);
        }
        if (out_f32)
            a4_launch_hn<_Float16, 2>(p, hn_tail, stream, wc, hn_level);
        else
            a4_launch_hn<_Float16, 1>(p, hn_tail, stream, wc, hn_level);
        return hipGetLastError();
    }
#endif
    a4_split_plan(p, ntiles, p.Kp / GK);
    const bool split = p.sk_split > 1;
    const int nunits = split ? p.sk_full + p.sk_split * p.sk_left : ntiles;
    const int ncu = a4_cus();
    const bool walk = walk_mode > 0 && (p.R != nullptr || walk_mode == 2) && ncu > 0 && nunits > ncu;
    const dim3 grid(walk ? ncu : nunits);
#ifdef VP3D_ABLATION
    static const int abl = [] {
        const char* e = getenv("VP3D_ABL");
        return e ? atoi(e) : 0;
    }();
    if (abl && !out_f32 && !split) {
        switch (abl) {
            case 1: a4_x3_abl<1>(p, grid); break;
            case 2: a4_x3_abl<2>(p, grid); break;
            case 3: a4_x3_abl<3>(p, grid); break;
            case 8: a4_x3_abl<8>(p, grid); break;
            case 16: a4_x3_abl<16>(p, grid); break;
            case 24: a4_x3_abl<24>(p, grid); break;
            case 32: a4_x3_abl<32>(p, grid); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
#endif
    if (out_f32)
        a4_launch<_Float16, 2>(p, grid, split, stream);
    else
        a4_launch<_Float16, 1>(p, grid, split, stream);
    return hipGetLastError();
}

hipError_t launch_conv_gemm_a4(const ConvGemmParams& p_in, Act compute, hipStream_t stream) {
    const int ntiles = ((p_in.M + GM - 1) / GM) * (p_in.N / GN);
    // Tile walk (one workgroup per CU; a multiple of 8 keeps each workgroup on one XCD's tile
    // range under round-robin placement) for the 1x1 + residual convs: the next tile's first
    // two K-tiles then land under this tile's epilogue and no workgroup launch gap separates
    // the tiles (B = 65,536, same box: block-1 1x1 3.69-3.70 vs 3.78-3.86 ms, blocks 2-4
    // -4..-8 %); the k3 convs keep one tile per workgroup (walked: the same or up to 2 %
    // slower).  With a residual the walk needs nk even (residual part h sits in the buffer
    // of the next tile's K-tile h; the split plan keeps every unit's nk even).  VP3D_A4_WALK
    // (measurement; read at every launch, so a test can flip it): 0 never, 2 every layer.
    const char* we = getenv("VP3D_A4_WALK");
    const int walk_mode = we ? atoi(we) : 1;
    const int ncu = a4_cus();
    const int nk = p_in.Kp / GK;
    ConvGemmParams p = p_in;
#ifndef VP3D_ABLATION
    const int hn_tail = walk_mode == 2 ? 0 : a4_hn_tail(p, ntiles, false);
    if (hn_tail > 0) {
        if (compute == Act::BF16)
            a4_launch_hn<__bf16, 0>(p, hn_tail, stream);
        else
            a4_launch_hn<_Float16, 0>(p, hn_tail, stream);
        return hipGetLastError();
    }
#endif
    {
        // a tail of <= a quarter round after whole rounds (sequence mode: 4 tiles past 4 rounds):
        // the whole rounds as the layer would run them, the tail split over every CU
        int lvl = 1;
        const int mt_tail = walk_mode == 2 ? 0 : a4_hn_tail(p, ntiles, true, &lvl);  // (the f16x3 tail shape)
        if (mt_tail > 0 && a4_tail_split(p, mt_tail, lvl, true)) {
            const int mt0 = (p.M + GM - 1) / GM - mt_tail;
            const int tiles = mt0 * (p.N / GN);
            const bool wk = walk_mode > 0 && p.R != nullptr && ncu > 0 && nk >= 3 && tiles > ncu && nk % 2 == 0;
            ConvGemmParams q = p;
            q.M = mt0 * GM;
            q.sk_split = q.sk_full = q.sk_left = 0;
            if (compute == Act::BF16)
                a4_launch<__bf16, 0>(q, dim3(wk ? ncu : tiles), false, stream);
            else
                a4_launch<_Float16, 0>(q, dim3(wk ? ncu : tiles), false, stream);
            return launch_conv_gemm_tail16(p, mt0 * GM, compute, ncu, stream);
        }
    }
    a4_split_plan(p, ntiles, nk);
    const bool split = p.sk_split > 1;
    const int nunits = split ? p.sk_full + p.sk_split * p.sk_left : ntiles;
    const bool walk = walk_mode > 0 && (p.R != nullptr || walk_mode == 2) && ncu > 0 && nk >= 3 && nunits > ncu &&
                      (!p.R || nk % 2 == 0);
    const dim3 grid(walk ? ncu : nunits);
#ifdef VP3D_ABLATION
    // measurement builds only (tools/ubench/gemm_check): VP3D_ABL=1 no loop DMA, 2 no loop
    // fragment reads, 3 neither (wrong results, timing only), 4 stamps
    static const int abl = [] {
        const char* e = getenv("VP3D_ABL");
        return e ? atoi(e) : 0;
    }();
    if (compute == Act::BF16 && abl >= 1) {
        p.sk_split = 0;
        const dim3 g(walk ? ncu : ntiles);
        switch (abl) {
            case 1: hipLaunchKernelGGL((conv_gemm_a4<__bf16, 1>), g, dim3(256), 0, stream, p); break;
            case 2: hipLaunchKernelGGL((conv_gemm_a4<__bf16, 2>), g, dim3(256), 0, stream, p); break;
            case 3: hipLaunchKernelGGL((conv_gemm_a4<__bf16, 3>), g, dim3(256), 0, stream, p); break;
            case 64: hipLaunchKernelGGL((conv_gemm_a4<__bf16, 64>), g, dim3(256), 0, stream, p); break;
            case 65: hipLaunchKernelGGL((conv_gemm_a4<__bf16, 65>), g, dim3(256), 0, stream, p); break;
            case 66: hipLaunchKernelGGL((conv_gemm_a4<__bf16, 66>), g, dim3(256), 0, stream, p); break;
            default: hipLaunchKernelGGL((conv_gemm_a4<__bf16, 4>), g, dim3(256), 0, stream, p); break;
        }
        return hipGetLastError();
    }
#endif
    if (compute == Act::BF16)
        a4_launch<__bf16, 0>(p, grid, split, stream);
    else
        a4_launch<_Float16, 0>(p, grid, split, stream);
    return hipGetLastError();
}

}  // namespace vp3d
