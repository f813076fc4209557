// Expand convolution of the lifter, 16-bit path, fused with the input packing.
//
// Reference: expand_conv + expand_bn + ReLU (+ dropout, identity in eval),
// common/models/TemporalModel.py:102,127 (TemporalModel) and :168,189
// (TemporalModelOptimized1f).  In channel-last layout output row m = (b, t) is
//   e[m, n] = relu(scale[n] * sum_k x[src(m)*lda + k] * W[n, k] + shift[n]),
//   src(m) = b*T_in + t*stride,  k < K = w0*J_in*F  (the w0 taps are contiguous frames)
// so every output row reads K contiguous f32 of the (B, T, J, F) input.
//
// Why a kernel of its own: K is tiny (102, or 138 with the camera concat) and
// N = 1024, so the layer is bound by writing its (M x 1024) 16-bit output, not by
// MFMA.  Here:
//   * A (the input rows) is read once, straight from the f32 input into MFMA
//     fragments in VGPRs (8-byte loads, converted to bf16/f16 in registers): no
//     packed copy in HBM, no A in LDS;
//   * one workgroup (4 waves) owns 64*RB rows and sweeps all N = 1024 output
//     channels in chunks of 64; the weights (<= 320 KB, L2-resident) stream through a
//     3-deep LDS ring of chunks, filled by LDS-DMA two chunks ahead (no VGPR staging);
//   * the eval BatchNorm is folded into the 16-bit weights the host prepares for this
//     kernel (Layer::wfbf / wfh: W * scale rounded once, shift as two 16-bit columns
//     hi + lo at k = K, K + 1 that the loader feeds with 1.0), so the epilogue is a
//     packed convert + a packed integer max for the ReLU (16-bit floats order like
//     sign-magnitude integers: max(bits, 0) is relu, -0 included) -- 1 VALU op per
//     output instead of 3.5 (scale, shift, max, convert: the old epilogue cost 0.6 ms
//     of 3.1 at B = 65,536; with no stores at all the old kernel still took 2.9 ms);
//   * the MFMA is issued transposed (D = W . A^T), so each lane's accumulator holds 4
//     consecutive channels of one row; they go to a wave-private LDS tile and out as
//     16-byte stores of whole 128-byte lines (8 rows x 128 B per instruction);
//   * the chunk loop ends on a raw barrier with a counted vmcnt (the weight DMA of the
//     next chunk only): the output stores stay in flight across chunks.
#include <cstdlib>

#include "gemm_common.h"

namespace vp3d {
namespace {

using namespace gemm;

constexpr int kExpWaves = 4;
constexpr int kExpChunkN = 64;  // output channels per chunk
constexpr int kExpMaxN = 1024;
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;
constexpr int kExpSlab = 4096;  // bytes of one [64 channels][32 k] slab
#ifdef VP3D_ABLATION
__device__ int g_expand_abl;
#endif

// two f32 -> two 16-bit floats (round to nearest even) in one dword, element 0 low:
// one v_cvt_pk_{bf16,f16}_f32 (compiler-generated, so the MFMA-result read hazard is
// handled by the compiler)
template <typename CT>
__device__ __forceinline__ uint32_t cvt_pk(float a, float b) {
    typedef float float2v __attribute__((ext_vector_type(2)));
    typedef CT ct2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(float2v{a, b}, ct2));
}

template <int N>
__device__ __forceinline__ void exp_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// RB = row blocks of 16 per wave (64 * RB rows per workgroup).
// GATHER: the input rows are not a (B, T, Cin) tensor but windows of device-resident
// sequences, gathered here (GatherSrc, kernels.h): the ChunkedGenerator batch and the
// camera concat fused into the operand loader.
// LDS image of a weight chunk: NKS slabs of [64 channels][32 k] (64-byte rows); the
// 16-byte unit c' of row r holds k-chunk (c' - 2 ((r >> 2) & 3)) & 3, so the fragment
// reads (row l & 15 of a 16-row block, k-chunk l >> 4) are bank-conflict free.  The DMA
// writes a slab lane-linearly (wave w: rows 16w .. 16w + 15); the permutation is applied
// to the global source address.
// RING: weight chunks resident (3: current, next, next-but-one; 2: current, next)
// X3 (split fp16, VP3D_DTYPE_F16X3; CT = f16): the f32 input rows are split in registers
// into hi = f16(x) and lo = f16(x - hi) fragments; the weights are Layer::wx3 (W 2^e as hi
// and lo halves, each 32-wide K group [hi(32) | lo(32)], BN NOT folded), so a weight chunk
// is 2 NKS slabs (hi, lo per k-slab) and each k-slab issues hi.hi + hi.lo + lo.hi; the
// epilogue applies the BatchNorm as ATen does (x * scale, then + shift, two roundings) +
// ReLU in the accumulator layout, then (as gemm::epilogue_tp) one v_permlane16_swap per
// value pair gives each lane 8 consecutive channels of a row, stored straight from
// registers as 16 bytes of hi and 16 of lo (channel n at 64 (n / 32) + n % 32 of the split
// row, lo 32 further): no LDS staging, so with a 2-chunk weight ring two workgroups share
// a CU and one's epilogue runs under the other's MFMAs.
// RING 1 (X3 only; round 6, the gathered NKS <= 4 shape): one weight chunk resident (32 KB + 8 KB
// of scale / shift) and RB 2 (154 VGPRs): three workgroups per CU instead of two, each staging its
// next chunk after the barrier that ends the current one and waiting for it (with the previous
// chunk's stores: vmcnt retires in order) -- the other two workgroups keep the CU busy meanwhile.
template <typename CT, int NKS, int RB, bool GATHER, bool NT = false, int RING = 3, bool X3 = false>
__global__ __launch_bounds__(256, (X3 && RING == 1) ? 3 : 2) void expand_gemm_h16(ConvGemmParams p, GatherSrc g) {
    constexpr int kRowsW = 16 * RB;
    constexpr int kRows = kRowsW * kExpWaves;
    constexpr int NKW = X3 ? 2 * NKS : NKS;  // weight slabs per chunk
    constexpr int kChunk = NKW * kExpSlab;
    // X3 with NKS = 5 (the camera concat): the 2 x 40 KB weight ring alone fills half the LDS, so
    // the scale / shift rows are read from global memory per chunk (ahead of its weight DMA)
    // instead of an 8 KB LDS copy -- two workgroups per CU instead of one
    constexpr bool kSsLds = !(X3 && NKS > 4);
    // ring of weight chunks, then (16-bit) per-wave output staging: kRowsW rows x 128 B,
    // 16-byte unit c of row r at c ^ (r & 7); X3: scale, shift (N floats each) instead
    __shared__ __attribute__((aligned(16))) char smem[RING * kChunk +
                                                      (X3 ? (kSsLds ? 2 * kExpMaxN * 4 : 0) : kExpWaves * kRowsW * 128)];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    // workgroups [0, sk_full): a whole row block each; after them each remaining row block is
    // sk_split workgroups of an equal channel-chunk range (the launcher's fill of the partial
    // last round, dispatched last)
    const int nchunks = p.N / kExpChunkN;
    int rblk = blockIdx.x, ch_lo = 0, ch_hi = nchunks;
    if (rblk >= p.sk_full) {
        const int u = rblk - p.sk_full, part = u % p.sk_split;
        rblk = p.sk_full + u / p.sk_split;
        ch_lo = part * nchunks / p.sk_split;
        ch_hi = (part + 1) * nchunks / p.sk_split;
    }
    const int m_wave = rblk * kRows + wid * kRowsW;
    // X3: this wave's output rows as a buffer resource (rows past M outside its range)
    __amdgpu_buffer_rsrc_t y_rsrc;
    if constexpr (X3) {
        const int mw = __builtin_amdgcn_readfirstlane(m_wave);  // wave-uniform: an SGPR resource
        const int64_t rows = p.M > mw ? (int64_t)(p.M - mw) : 0;
        y_rsrc = make_rsrc((const char*)((const f16*)p.Y + (int64_t)mw * p.ldy), clamp_range31((size_t)rows * p.ldy * 2));
    }
    u32x4* const stage = (u32x4*)(smem + RING * kChunk + wid * kRowsW * 128);
    float* const s_scale = (float*)(smem + RING * kChunk);
    float* const s_shift = s_scale + kExpMaxN;
    if constexpr (X3 && kSsLds) {
        for (int i = tid; i < p.N; i += 256) {
            s_scale[i] = p.scale[i];
            s_shift[i] = p.shift[i];
        }
    }

    // ---- weight chunk DMA: NKS pieces of 1 KB per wave ----
    const int dr = 16 * wid + (lane >> 2);
    const int dc = ((lane & 3) - 2 * ((dr >> 2) & 3)) & 3;
    const CT* const wsrc = (const CT*)p.W + (int64_t)dr * p.Kp + dc * 8;
    auto stage_w = [&](int chunk) {
        char* dst = smem + ((chunk - ch_lo) % RING) * kChunk + wid * 1024;
        const CT* src = wsrc + (int64_t)chunk * kExpChunkN * p.Kp;
#pragma unroll
        for (int q = 0; q < NKW; ++q)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src + q * 32), (lds_ptr_t)(dst + q * kExpSlab), 16, 0, 0);
    };
    stage_w(ch_lo);
    if (RING == 3 && ch_lo + 1 < ch_hi) stage_w(ch_lo + 1);

    // ---- A fragments: row (l & 15) of each 16-row block, k = 32*ks + 8*(l>>4) .. +7;
    // k = K, K + 1 are the bias columns (1.0), k > K + 1 zero ----
    const float* X = (const float*)p.A;
    u32x4 af[RB][NKS];
    u32x4 afl[X3 ? RB : 1][NKS];  // X3: the lo fragments
    constexpr float kBias = X3 ? 0.f : 1.f;  // the folded-shift column (16-bit path only)
    uint32_t x_hmax = 0;  // X3: max |hi| bits of the input rows (gemm::x3_hi_bad: inf / NaN)
    auto put = [&](int rb, int ks, const float (&v)[8]) {
        if constexpr (X3) {
            f16x8 h, l;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                h[e] = (f16)v[e];
                l[e] = (f16)(v[e] - (float)h[e]);
            }
            const u32x4 hw = __builtin_bit_cast(u32x4, h);
#pragma unroll
            for (int e = 0; e < 4; ++e) x_hmax = gemm::x3_himax2(x_hmax, hw[e]);
            af[rb][ks] = __builtin_bit_cast(u32x4, h);
            afl[rb][ks] = __builtin_bit_cast(u32x4, l);
        } else {
            af[rb][ks] = pack8<CT>(v);
        }
    };
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
        int m = m_wave + rb * 16 + (lane & 15);
        m = m < p.M ? m : p.M - 1;  // rows past M read a valid row; never stored
        if constexpr (!GATHER) {
            const float* row = X + (int64_t)src_row(p, m) * p.lda;
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const int k0 = ks * 32 + (lane >> 4) * 8;
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; e += 2) {
                    // K even: pairs are wholly in or out; out-of-range pairs read pair 0
                    const bool in = k0 + e < p.K;
                    const float t = k0 + e == p.K ? kBias : 0.f;
                    const float2 x = *(const float2*)(row + (in ? k0 + e : 0));
                    v[e] = in ? x.x : t;
                    v[e + 1] = in ? x.y : t;
                }
                put(rb, ks, v);
            }
        } else {
            // window b starts at sequence frame start_b - lead; row t covers window frames
            // t*stride + tap, tap < K / lda; frame j of the window is sequence frame
            // clamp(start_b - lead + j, 0, len - 1) ('edge' padding, generators.py:92-100)
            const int b = m / p.T_out;
            const int t = m - b * p.T_out;
            const int2 pr = *(const int2*)(g.pairs + 2 * b);
            const int64_t off = g.seq_off[pr.x];
            const int len = g.seq_len[pr.x];
            const int f0 = pr.y - g.lead + t * p.stride;
            // no camera concat and no clamped frame in the row (the common case): the
            // row's K values are contiguous in the sequence, one base address per row.
            // Only the last k-slab holds k >= K (K + 2 > 32 (NKS - 1) and K even).
            const bool flat = g.cams == nullptr && f0 >= 0 && f0 + p.K / p.lda <= len;
            if (__all(flat)) {
                const float* row = g.kps + (off + f0) * g.f2;
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) {
                    const int k0 = ks * 32 + (lane >> 4) * 8;
                    float v[8];
#pragma unroll
                    for (int e = 0; e < 8; e += 2) {
                        const int k = k0 + e;
                        if (ks + 1 < NKS) {
                            const float2 x = *(const float2*)(row + k);
                            v[e] = x.x;
                            v[e + 1] = x.y;
                        } else {
                            const bool in = k < p.K;
                            const float t1 = k == p.K ? kBias : 0.f;
                            const float2 x = *(const float2*)(row + (in ? k : 0));
                            v[e] = in ? x.x : t1;
                            v[e + 1] = in ? x.y : t1;
                        }
                    }
                    put(rb, ks, v);
                }
                continue;
            }
            // tap = k / lda without an integer division: k < 2^12 and lda <= 2^11, so
            // (k + 0.5) * (1 / lda) stays > 1/(4 lda) away from the next integer
            const float inv_lda = 1.0f / (float)p.lda;
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const int k0 = ks * 32 + (lane >> 4) * 8;
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; e += 2) {
                    // lda, f2 and K even: a pair never straddles a tap or the kps|cams edge
                    const int k = k0 + e;
                    const bool in = k < p.K;
                    const float t1 = k == p.K ? kBias : 0.f;
                    const int tap = in ? (int)(((float)k + 0.5f) * inv_lda) : 0;
                    const int c = in ? k - tap * p.lda : 0;
                    int fr = f0 + tap;
                    fr = fr < 0 ? 0 : (fr >= len ? len - 1 : fr);
                    const int64_t gf = off + fr;
                    const float* src = c < g.f2 ? g.kps + gf * g.f2 + c : g.cams + gf * 12 + (c - g.f2);
                    const float2 tv = *(const float2*)src;
                    v[e] = in ? tv.x : t1;
                    v[e + 1] = in ? tv.y : t1;
                }
                put(rb, ks, v);
            }
        }
    }
    exp_vm<0>();  // weight chunks 0 and 1 (and the A loads) landed
    __builtin_amdgcn_s_barrier();
    if constexpr (X3) gemm::x3_range_flag(gemm::x3_hi_bad(x_hmax) ? __builtin_inff() : 0.f, p.scale, p.N);

#ifdef VP3D_ABLATION
    // measurement builds only (tools/ubench/expand_check): 2 = no global stores,
    // 4 = no wait for the next weight chunk (results wrong; timing only)
    const int abl = g_expand_abl;
#else
    constexpr int abl = 0;
#endif
    const int frag_off = ((lane & 15) * 4 + (((lane >> 4) + 2 * (((lane & 15) >> 2) & 3)) & 3)) * 16;
    CT* Y = (CT*)p.Y;
    typedef short short2v __attribute__((ext_vector_type(2)));
    // ReLU on the packed 16-bit results: max with +0 (bits 0); no ReLU: max with the
    // smallest int16, a no-op
    const short2v floor2 = p.relu ? short2v{0, 0} : short2v{-32768, -32768};
    for (int ch = ch_lo; ch < ch_hi; ++ch) {
        // chunk ch + 2 goes to the slot chunk ch - 1 used: every wave passed the barrier
        // that ended chunk ch - 1 after its last fragment read there
        f32x4 gs4[kSsLds ? 1 : 4], gh4[kSsLds ? 1 : 4];  // !kSsLds: this chunk's scale / shift
        if constexpr (!kSsLds) {
            const int gc = ch * kExpChunkN + 4 * (lane >> 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                gs4[j] = *(const f32x4*)(p.scale + gc + 16 * j);
                gh4[j] = *(const f32x4*)(p.shift + gc + 16 * j);
            }
        }
        if constexpr (RING == 1) {
            // the single slot: every wave passed the barrier that ended chunk ch - 1
            if (ch > ch_lo) {
                stage_w(ch);
                exp_vm<0>();
                __builtin_amdgcn_s_barrier();
            }
        } else if (ch + RING - 1 < ch_hi) {
            stage_w(ch + RING - 1);
        }
        const char* wb = smem + ((ch - ch_lo) % RING) * kChunk;
        f32x4 acc[RB][4];
        if constexpr (X3) {
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                u32x4 wh[4], wl[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    wh[j] = *(const u32x4*)(wb + (2 * ks) * kExpSlab + j * 1024 + frag_off);
                    wl[j] = *(const u32x4*)(wb + (2 * ks + 1) * kExpSlab + j * 1024 + frag_off);
                }
                if (abl & 16) {  // (measurement builds: no MFMAs -- the store stream alone)
#pragma unroll
                    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            acc[rb][j] = f32x4{__builtin_bit_cast(float, wh[j][0] ^ af[rb][ks][0]), 0.f, 0.f, 0.f};
                    continue;
                }
#pragma unroll
                for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[rb][j] = mfma16<CT>(wh[j], af[rb][ks], ks == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[rb][j]);
#pragma unroll
                for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[rb][j] = mfma16<CT>(wh[j], afl[rb][ks], acc[rb][j]);
#pragma unroll
                for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[rb][j] = mfma16<CT>(wl[j], af[rb][ks], acc[rb][j]);
            }
            // epilogue: BN affine (two roundings) + ReLU in the accumulator layout (lane: channels
            // n0 + 16 j + 4 (l >> 4) + r of row 16 rb + (l & 15)); the permlane swap pairs j = 2 jp,
            // 2 jp + 1 so each lane then holds channels n0 + 32 jp + c0 + 0..7 of its row
            const int n0 = ch * kExpChunkN;
            const int grp = lane >> 4;
            const int c0 = 8 * ((grp & 1) * 2 + (grp >> 1));
            typedef float f32x2 __attribute__((ext_vector_type(2)));
            typedef int i32x2 __attribute__((ext_vector_type(2)));
            f32x2 sc[4][2], sh[4][2];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                f32x4 s4, h4;
                if constexpr (kSsLds) {
                    s4 = *(const f32x4*)&s_scale[n0 + 16 * j + 4 * grp];
                    h4 = *(const f32x4*)&s_shift[n0 + 16 * j + 4 * grp];
                } else {
                    s4 = gs4[j];
                    h4 = gh4[j];
                }
                sc[j][0] = f32x2{s4[0], s4[1]};
                sc[j][1] = f32x2{s4[2], s4[3]};
                sh[j][0] = f32x2{h4[0], h4[1]};
                sh[j][1] = f32x2{h4[2], h4[3]};
            }
            const int r16 = lane & 15;
            const bool top = r16 < 8;
            float vmax = 0.f;  // |x| over what this chunk splits (gemm::x3_range_flag)
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
                for (int jp = 0; jp < 2; ++jp) {
                    // BN affine as ATen forms it (x * scale, then + shift: two roundings, packed
                    // v_pk_mul_f32 / v_pk_add_f32) + ReLU as an integer max on the f32 bits
                    // (negative and -0 -> +0, as x > 0 ? x : 0) in the accumulator layout (lane:
                    // channels n0 + 16 j + 4 (l >> 4) + 0..3 of row 16 rb + (l & 15))
                    float x[4], y[4];
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
#pragma unroll
                        for (int hp = 0; hp < 2; ++hp) {
                            const int j = 2 * jp + q;
                            f32x2 t = f32x2{acc[rb][j][2 * hp], acc[rb][j][2 * hp + 1]} * sc[j][hp];
                            t = t + sh[j][hp];
                            i32x2 ti = __builtin_bit_cast(i32x2, t);  // (the X3 expand is always BN + ReLU)
                            ti = __builtin_elementwise_max(ti, i32x2{0, 0});
                            t = __builtin_bit_cast(f32x2, ti);
                            float* d = q ? y : x;
                            d[2 * hp] = t[0];
                            d[2 * hp + 1] = t[1];
                        }
                    }
                    // blocks 2 jp, 2 jp + 1 -> 8 consecutive channels n0 + 32 jp + c0 + 0..7 per
                    // lane (the x values just written by VALU: 2 wait states before the swaps)
                    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\tv_permlane16_swap_b32 %2, %3\n\t"
                                 "v_permlane16_swap_b32 %4, %5\n\tv_permlane16_swap_b32 %6, %7"
                                 : "+v"(x[0]), "+v"(y[0]), "+v"(x[1]), "+v"(y[1]), "+v"(x[2]), "+v"(y[2]),
                                   "+v"(x[3]), "+v"(y[3]));
                    const float v[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
                    // hi = f16(v), lo = f16(v - hi) (v_fma_mixlo/mixhi: one rounding each)
                    u32x4 oh, ol;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        oh[e] = gemm::x3_hi2(v[2 * e], v[2 * e + 1]);
                        ol[e] = gemm::x3_split_lo2(oh[e], v[2 * e], v[2 * e + 1]);
                        vmax = gemm::x3_absmax2(vmax, v[2 * e], v[2 * e + 1]);
                    }
                    // (the camera-concat shape too since round 5: it had kept half lines of 16 rows
                    // per instruction, nontemporal; whole lines at 3 row blocks per wave: config-3
                    // expand 6.24-6.25 vs 6.37-6.40 ms, profiles/r05_x3_expand_rb_policy_ab.txt)
                    // whole 128-byte lines per store instruction: the line of row r holds its 32
                    // hi then 32 lo channels; lanes of rows 8-15 of the 16 trade with rows 0-7 (DPP
                    // row_ror:8, written only into the bank half that takes the partner's value)
                    // so instruction A writes rows 0-7 (hi from lanes 0-7, lo from lanes 8-15) and
                    // instruction B rows 8-15 -- instead of two 64-byte halves of 16 lines (config
                    // 4, B = 65,536: 5.24-5.26 vs 5.64-5.72 ms, profiles/r04final_x3_expand_whole_lines_ab.txt)
                    u32x4 va, vb;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        va[e] = (uint32_t)__builtin_amdgcn_update_dpp((int)oh[e], (int)ol[e], 0x128, 0xF, 0xC, false);
                        vb[e] = (uint32_t)__builtin_amdgcn_update_dpp((int)ol[e], (int)oh[e], 0x128, 0xF, 0x3, false);
                    }
                    if (abl & 2) {  // (measurement builds: no output stores)
                        asm volatile("" ::"v"(va), "v"(vb));
                        continue;
                    }
                    // buffer stores through the wave's own resource (rows past M fall outside it:
                    // no exec-mask branches per store)
                    const int ra = top ? r16 : r16 - 8, rbw = top ? r16 + 8 : r16;
                    const int half = top ? 0 : 32;  // lo 64 bytes further
                    const uint32_t oa = (uint32_t)(((rb * 16 + ra) * p.ldy + 2 * n0 + 64 * jp + c0 + half) * 2);
                    const uint32_t ob = (uint32_t)(((rb * 16 + rbw) * p.ldy + 2 * n0 + 64 * jp + c0 + half) * 2);
                    __builtin_amdgcn_raw_buffer_store_b128(va, y_rsrc, oa, 0, NT ? 2 : 0);
                    __builtin_amdgcn_raw_buffer_store_b128(vb, y_rsrc, ob, 0, NT ? 2 : 0);
                }
            }
            gemm::x3_range_flag(vmax, p.scale, p.N);
            asm volatile("" ::: "memory");
            if (RING > 1 && ch + 1 < ch_hi && !(abl & 4)) {
                if (m_wave + kRowsW > p.M || (abl & 2))
                    exp_vm<0>();
                else if (RING == 3 && ch + 2 < ch_hi)
                    exp_vm<NKW + 4 * RB>();
                else
                    exp_vm<4 * RB>();  // this chunk's stores: RB row blocks x 2 channel halves x (hi, lo)
            }
            __builtin_amdgcn_s_barrier();
            continue;
        }
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            u32x4 wf[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) wf[j] = *(const u32x4*)(wb + ks * kExpSlab + j * 1024 + frag_off);
#pragma unroll
            for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[rb][j] = mfma16<CT>(wf[j], af[rb][ks], ks == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[rb][j]);
        }

        // epilogue: lane holds channels n0 + 16j + 4(l>>4) + r of row rb*16 + (l & 15)
        const int n0 = ch * kExpChunkN;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int nl = j * 16 + (lane >> 4) * 4;  // channel within the chunk
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) {
                const short2v l2 = __builtin_elementwise_max(
                    __builtin_bit_cast(short2v, cvt_pk<CT>(acc[rb][j][0], acc[rb][j][1])), floor2);
                const short2v h2 = __builtin_elementwise_max(
                    __builtin_bit_cast(short2v, cvt_pk<CT>(acc[rb][j][2], acc[rb][j][3])), floor2);
                const int row = rb * 16 + (lane & 15);
                const int c16 = nl >> 3;  // 16-byte unit (8 channels), half (nl >> 2) & 1
                // the half is swapped on rows 8-15 of each 16: the 16 lanes of a write group
                // then cover all 32 banks (rows r and r + 8 otherwise shared them)
                char* dst = (char*)stage + row * 128 + ((c16 ^ (row & 7)) << 4) +
                            ((((nl >> 2) & 1) ^ ((row >> 3) & 1)) << 3);
                *(uint2*)dst = uint2{__builtin_bit_cast(uint32_t, l2), __builtin_bit_cast(uint32_t, h2)};
            }
        }
        asm volatile("" ::: "memory");
        // 8 lanes per row, 8 rows per instruction: whole 128-byte lines
#pragma unroll
        for (int q = 0; q < 2 * RB; ++q) {
            const int row = q * 8 + (lane >> 3);
            const int c16 = lane & 7;
            u32x4 v = stage[row * 8 + (c16 ^ (row & 7))];
            if (q & 1) v = u32x4{v.z, v.w, v.x, v.y};  // rows 8-15 of 16: halves swapped
            const int m = m_wave + row;
            if (abl == 2) {
                asm volatile("" ::"v"(v));
            } else if (m < p.M) {
                u32x4* dst = (u32x4*)(Y + (int64_t)m * p.ldy + n0 + c16 * 8);
                if constexpr (NT)
                    __builtin_nontemporal_store(v, dst);
                else
                    *dst = v;
            }
        }
        asm volatile("" ::: "memory");
        // the next chunk's weights: younger are chunk ch + 2's DMA (if issued) and this
        // chunk's 2 * RB stores.  A wave with rows past M may skip store instructions
        // (all lanes masked): fewer younger operations, so it drains everything instead.
        if (ch + 1 < ch_hi && abl != 4) {
            if (m_wave + kRowsW > p.M || abl == 2)
                exp_vm<0>();
            else if (RING == 3 && ch + 2 < ch_hi)
                exp_vm<NKS + 2 * RB>();
            else
                exp_vm<2 * RB>();
        }
        __builtin_amdgcn_s_barrier();
    }
}

// resident workgroup slots per launch: two per CU (__launch_bounds__(256, 2)) for every
// variant -- the camera-concat NKS = 5 one included since its RB 4 / 2-chunk weight ring
// (72 KB of LDS)
static int exp_slots(int per_cu = 2) {
    static const int ncu = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 0;
        return n;
    }();
    return per_cu * ncu;
}

// One workgroup per row block, except in a partial last round: with L < slots row blocks
// past the last whole round (or in all, for small M), each is split into S = min(slots / L, 8) workgroups of 16 / S
// channel chunks (dispatched last), so that round takes 1 / S of a round's time
// (B = 8,192: the f16x3 expand is 10.1 rounds of 512 row blocks, the bf16 one 5.06).
// Measured there: expand 0.85 vs 0.87 ms (f16x3), 0.295 vs 0.305 ms (bf16), +0.3-0.6 % per
// step -- the memory-bound tail was already short, its few row blocks running with the
// whole chip's bandwidth (profiles/r04x_expand_split_round_ab.txt).
// VP3D_EXPAND_SPLIT=0 (measurement) keeps whole row blocks.
template <typename CT, int RB, bool GATHER, bool NT, int RING = 3, bool X3 = false>
hipError_t launch_rb_nt(const ConvGemmParams& p_in, const GatherSrc& g, int nks, hipStream_t s) {
    ConvGemmParams p = p_in;
    const int nrb = (p.M + 64 * RB - 1) / (64 * RB);
    const int slots = exp_slots((X3 && RING == 1) ? 3 : 2);
    const int left = slots > 0 ? nrb % slots : 0;
    int S = left > 0 ? slots / left : 1;
    S = S > 8 ? 8 : S;
    const int nchunks = p.N / kExpChunkN;
    while (S > 1 && nchunks % S) --S;
    const char* off = getenv("VP3D_EXPAND_SPLIT");  // read at every launch (the A/B tests flip it)
    if (off && off[0] == '0') S = 1;
    p.sk_full = S > 1 ? nrb - left : nrb;
    p.sk_split = S;
    const dim3 grid(p.sk_full + (S > 1 ? left * S : 0));
    switch (nks) {
        case 1: hipLaunchKernelGGL((expand_gemm_h16<CT, 1, RB, GATHER, NT, RING, X3>), grid, dim3(256), 0, s, p, g); break;
        case 2: hipLaunchKernelGGL((expand_gemm_h16<CT, 2, RB, GATHER, NT, RING, X3>), grid, dim3(256), 0, s, p, g); break;
        case 3: hipLaunchKernelGGL((expand_gemm_h16<CT, 3, RB, GATHER, NT, RING, X3>), grid, dim3(256), 0, s, p, g); break;
        case 4: hipLaunchKernelGGL((expand_gemm_h16<CT, 4, RB, GATHER, NT, RING, X3>), grid, dim3(256), 0, s, p, g); break;
        case 5: hipLaunchKernelGGL((expand_gemm_h16<CT, 5, RB, GATHER, NT, RING, X3>), grid, dim3(256), 0, s, p, g); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Output stores are nontemporal when the output exceeds the 256 MB Infinity Cache: the
// 1.36 GB output (B = 8192) cannot stay there anyway; streamed past it, it leaves the
// caches to the weights and the block-1 conv that follows runs 1-1.5 % faster (3.10-3.12
// vs 3.14-3.18 ms per step, A/B on one box).  A smaller output is left cached for the
// next layer.
//
// Row blocks of 16 per wave (RB): more rows per wave amortise each weight chunk's
// fragment reads and the per-workgroup prologue; LDS is 3 weight chunks + RB * 8 KB of
// output staging per workgroup, and 2 workgroups per CU need <= 80 KB.  RB = 4 for
// K + 2 <= 128 (80 KB, 196-209 VGPRs: 2 waves per SIMD); the camera concat (K = 138, 5
// k-slabs) RB = 4 with a 2-chunk ring (72 KB, 212 VGPRs): config-3 fp16 expand 2.30 vs 2.57 ms
// with RB 2 and 3 chunks (profiles/r04final_concat_expand_rb4_ab.txt).  Measured on the config-4 shape (B = 65,536 windows, gathered, bf16,
// tools/ubench/expand_check): RB 4 -> 2.07 ms, 2 -> 2.25, 1 -> 2.74; the previous
// kernel (BN in the epilogue, weights staged through VGPRs, a full drain per chunk)
// took 3.12 ms.
#ifdef VP3D_ABLATION
int g_expand_rb = 0;
#endif
template <typename CT, bool GATHER>
hipError_t launch_t(const ConvGemmParams& p, const GatherSrc& g, int nks, hipStream_t s) {
    const bool nt = (int64_t)p.M * p.ldy * 2 > (int64_t)256 << 20;
#ifdef VP3D_ABLATION
    if (g_expand_rb == 12)  // RB 2, double-buffered weights (3 workgroups per CU)
        return nt ? launch_rb_nt<CT, 2, GATHER, true, 2>(p, g, nks, s) : launch_rb_nt<CT, 2, GATHER, false, 2>(p, g, nks, s);
    if (g_expand_rb == 14)  // RB 4, double-buffered weights
        return nt ? launch_rb_nt<CT, 4, GATHER, true, 2>(p, g, nks, s) : launch_rb_nt<CT, 4, GATHER, false, 2>(p, g, nks, s);
    if (g_expand_rb == 1)
        return nt ? launch_rb_nt<CT, 1, GATHER, true>(p, g, nks, s) : launch_rb_nt<CT, 1, GATHER, false>(p, g, nks, s);
    if (g_expand_rb == 2)
        return nt ? launch_rb_nt<CT, 2, GATHER, true>(p, g, nks, s) : launch_rb_nt<CT, 2, GATHER, false>(p, g, nks, s);
    if (g_expand_rb == 4)
        return nt ? launch_rb_nt<CT, 4, GATHER, true>(p, g, nks, s) : launch_rb_nt<CT, 4, GATHER, false>(p, g, nks, s);
#endif
    if (nks <= 4)
        return nt ? launch_rb_nt<CT, 4, GATHER, true>(p, g, nks, s) : launch_rb_nt<CT, 4, GATHER, false>(p, g, nks, s);
    return nt ? launch_rb_nt<CT, 4, GATHER, true, 2>(p, g, nks, s) : launch_rb_nt<CT, 4, GATHER, false, 2>(p, g, nks, s);
}

}  // namespace

bool expand_gemm_eligible(const ConvGemmParams& p, Act out_type, Act compute) {
    if (compute == Act::F32 || out_type != compute) return false;
    if (p.Ktap != p.K || p.dil != 1) return false;  // taps collapsed into one contiguous K run
    const int nks = (p.K + 2 + 31) / 32;  // K data columns + the two bias columns
    if (nks < 1 || nks > 5 || nks * 32 > p.Kp) return false;  // K <= 158 (LDS for 2 WG/CU)
    if (p.K % 2 || p.lda % 2 || (reinterpret_cast<uintptr_t>(p.A) & 7)) return false;
    if (p.N % kExpChunkN || p.N > kExpMaxN || p.ldy % 8 || (reinterpret_cast<uintptr_t>(p.Y) & 15))
        return false;
    return p.R == nullptr && p.M > 0;
}

bool expand_gather_eligible(const ConvGemmParams& p, const GatherSrc& g, Act out_type, Act compute) {
    if (!expand_gemm_eligible(p, out_type, compute)) return false;
    if (g.f2 % 2 || (reinterpret_cast<uintptr_t>(g.kps) & 7) || (g.cams && (reinterpret_cast<uintptr_t>(g.cams) & 7)))
        return false;
    return p.lda == g.f2 + (g.cams ? 12 : 0);
}

hipError_t launch_expand_gemm(const ConvGemmParams& p, Act compute, hipStream_t stream) {
    const int nks = (p.K + 2 + 31) / 32;
    const GatherSrc none{};
    return compute == Act::BF16 ? launch_t<bf16, false>(p, none, nks, stream)
                                : launch_t<f16, false>(p, none, nks, stream);
}

hipError_t launch_expand_gemm_gather(const ConvGemmParams& p, const GatherSrc& g, Act compute,
                                     hipStream_t stream) {
    const int nks = (p.K + 2 + 31) / 32;
    return compute == Act::BF16 ? launch_t<bf16, true>(p, g, nks, stream) : launch_t<f16, true>(p, g, nks, stream);
}

// Split-fp16 expand (X3): p.W = Layer::wx3 with p.Kp its row pitch in halves (2 Kp), the
// scale / shift unfolded (scale_x3, shift), p.ldy the split output pitch in halves (2 N).
bool expand_gemm_x3_eligible(const ConvGemmParams& p, const GatherSrc* g) {
    if (p.Ktap != p.K || p.dil != 1 || p.relu != 1) return false;  // expand_bn + ReLU (TemporalModel.py:127,189)
    const int nks = (p.K + 31) / 32;
    if (nks < 1 || nks > 5 || 2 * nks * 32 > p.Kp) return false;
    if (p.K % 2 || p.lda % 2 || (!g && (reinterpret_cast<uintptr_t>(p.A) & 7))) return false;
    if (p.N % kExpChunkN || p.N > kExpMaxN || p.ldy % 8 || (reinterpret_cast<uintptr_t>(p.Y) & 15)) return false;
    if (g && (g->f2 % 2 || (reinterpret_cast<uintptr_t>(g->kps) & 7) ||
              (g->cams && (reinterpret_cast<uintptr_t>(g->cams) & 7)) || p.lda != g->f2 + (g->cams ? 12 : 0)))
        return false;
    return p.R == nullptr && p.M > 0;
}

hipError_t launch_expand_gemm_x3(const ConvGemmParams& p, const GatherSrc* g, hipStream_t stream) {
    const int nks = (p.K + 31) / 32;
    const bool nt = (int64_t)p.M * p.ldy * 2 > (int64_t)256 << 20;
    const GatherSrc none{};
    // RB 3 row blocks per wave (each weight chunk staged into LDS serves 192 rows instead of
    // 128), 2-chunk weight ring: 2 x 32 KB + 8 KB scale / shift (NKS 4), two workgroups per
    // CU (206 / 250 VGPRs at NKS 4 / 5; RB 4 spills).  Same box vs RB 2: config-3 expand (the
    // camera concat, NKS 5) 6.43-6.46 vs 6.75 ms, config 4 within noise; forwards
    // bit-identical (profiles/r05_x3_expand_rb3_ab.txt)
    // RB 3 or 2 by the rounds each leaves (a partial last round of few row blocks is split
    // into channel-range workgroups, launch_rb_nt): per-round cost ~ RB, the last round costs
    // 1 / S of a round -- 8,192 windows: RB 2 (10 rounds + 1/8) over RB 3 (6 + a 0.75 round)
    const int slots = exp_slots();
    auto cost = [&](int rb) {
        const int nrb = (p.M + 64 * rb - 1) / (64 * rb);
        if (slots <= 0) return (double)nrb * rb;
        const int full = nrb / slots, left = nrb % slots;
        int S = left > 0 ? slots / left : 1;
        S = S > 8 ? 8 : S;
        return (full + (left > 0 ? 1.0 / S : 0.0)) * rb;
    };
    const bool rb3 = cost(3) <= cost(2) + 1e-9;
    // the gathered config-2/4 shape (K = 102, NKS 4): three workgroups per CU (RING 1, RB 2:
    // 40 KB of LDS, 154 VGPRs) -- config 4 expand 5.18-5.21 vs 5.30-5.31 ms at B = 65,536, 0.698-0.702
    // vs 0.703-0.705 at 8,192, same box, forwards bit-identical (profiles/r06_x3_expand_ring1_ab.txt);
    // VP3D_X3_EXPAND_RING=2 (measurement, read at every launch) keeps the two-per-CU form below
    const char* ring = getenv("VP3D_X3_EXPAND_RING");
    if (!(ring && ring[0] == '2') && g && nks <= 4)
        return nt ? launch_rb_nt<f16, 2, true, true, 1, true>(p, *g, nks, stream)
                  : launch_rb_nt<f16, 2, true, false, 1, true>(p, *g, nks, stream);
    if (g) {
        if (rb3)
            return nt ? launch_rb_nt<f16, 3, true, true, 2, true>(p, *g, nks, stream)
                      : launch_rb_nt<f16, 3, true, false, 2, true>(p, *g, nks, stream);
        return nt ? launch_rb_nt<f16, 2, true, true, 2, true>(p, *g, nks, stream)
                  : launch_rb_nt<f16, 2, true, false, 2, true>(p, *g, nks, stream);
    }
    return nt ? launch_rb_nt<f16, 2, false, true, 2, true>(p, none, nks, stream)
              : launch_rb_nt<f16, 2, false, false, 2, true>(p, none, nks, stream);
}

}  // namespace vp3d

#ifdef VP3D_ABLATION
namespace vp3d {
hipError_t expand_gemm_set_ablation(int a) { return hipMemcpyToSymbol(HIP_SYMBOL(g_expand_abl), &a, sizeof(int)); }
void expand_gemm_set_rb(int rb) { g_expand_rb = rb; }
}  // namespace vp3d
#endif
