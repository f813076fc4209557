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
// MFMA.  The generic path (pack f32 rows to padded 16-bit rows, then a 256x256
// GEMM with 4 K-steps) spent ~0.75 ms at B = 8192 on what is ~1.6 GB of HBM
// traffic.  Here:
//   * A (the input rows) is read once, straight from the f32 input into MFMA
//     fragments in VGPRs (8-byte loads, converted to bf16/f16 in registers): no
//     packed copy in HBM, no A in LDS;
//   * one workgroup (4 waves) owns 256 rows and sweeps all N = 1024 output
//     channels in chunks of 64; the weights (<= 384 KB, L2-resident) stream
//     through a double-buffered LDS chunk shared by the 4 waves;
//   * the MFMA is issued transposed (D = W . A^T: v_mfma_f32_16x16x32 with the
//     weight fragment as the A operand), so each lane's accumulator holds 4
//     consecutive channels of one row: BN affine + ReLU + 16-bit convert in
//     registers, one 8-byte write per (row block, channel block) into a
//     wave-private LDS tile, then 16-byte stores of whole 128-byte lines
//     (8 rows x 128 B per instruction).  The store path, not the MFMA, sets this
//     kernel's speed: with 8-byte stores straight from the accumulators (16 rows
//     x 32 B per instruction) the TA was busy 80 % of the kernel at ~120 cycles
//     per store instruction (rocprofv3 TA_BUSY / TA_FLAT_WRITE_WAVEFRONTS).
#include <cstdlib>

#include "gemm_common.h"

namespace vp3d {
namespace {

using namespace gemm;

constexpr int kExpWaves = 4;
constexpr int kExpChunkN = 64;                          // output channels per chunk
constexpr int kExpMaxN = 1024;

// LDS layout of one weight chunk: NKS slabs of [64 channels][32 k] (64-byte rows),
// 16-byte chunk c of row r stored at chunk (c + 2*((r>>2)&3)) & 3 -> the fragment
// reads (row l&15 of a 16-row block, chunk l>>4) are bank-conflict free.
__device__ __forceinline__ int exp_swz(int r, int c) { return r * 4 + ((c + 2 * ((r >> 2) & 3)) & 3); }

// RB = row blocks of 16 per wave (64 * RB rows per workgroup).
// GATHER: the input rows are not a (B, T, Cin) tensor but windows of device-resident
// sequences, gathered here (GatherSrc, kernels.h): the ChunkedGenerator batch and the
// camera concat fused into the operand loader.
template <typename CT, int NKS, int RB, bool GATHER, bool NT = false>
__global__ __launch_bounds__(256) void expand_gemm_h16(ConvGemmParams p, GatherSrc g) {
    constexpr int kExpRowsPerWave = 16 * RB;
    constexpr int kExpRows = kExpRowsPerWave * kExpWaves;
    constexpr int SLAB = kExpChunkN * 4;       // 16-byte units per k-step slab
    constexpr int CHUNK_U = NKS * SLAB;        // 16-byte units per weight chunk
    __shared__ __attribute__((aligned(16))) u32x4 wbuf[2][CHUNK_U];
    __shared__ __attribute__((aligned(16))) float s_scale[kExpMaxN];
    __shared__ __attribute__((aligned(16))) float s_shift[kExpMaxN];
    // per-wave output staging: 64 rows x 128 B, 16-byte chunk c of row r at c ^ (r & 7)
    __shared__ __attribute__((aligned(16))) u32x4 s_out[kExpWaves][kExpRowsPerWave * 8];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int m_wave = blockIdx.x * kExpRows + wid * kExpRowsPerWave;

    for (int i = tid; i < p.N; i += 256) {
        s_scale[i] = p.scale[i];
        s_shift[i] = p.shift[i];
    }

    // ---- weight chunk staging: NKS 16-byte pieces per thread ----
    const CT* W = (const CT*)p.W;
    const int st_row = tid >> 2, st_c = tid & 3;
    u32x4 wst[NKS];
    auto wload = [&](int chunk) {
        const CT* src = W + (int64_t)(chunk * kExpChunkN + st_row) * p.Kp + st_c * 8;
#pragma unroll
        for (int q = 0; q < NKS; ++q) wst[q] = *(const u32x4*)(src + q * 32);
    };
    auto wstore = [&](int buf) {
#pragma unroll
        for (int q = 0; q < NKS; ++q) wbuf[buf][q * SLAB + exp_swz(st_row, st_c)] = wst[q];
    };

    // ---- A fragments: row (l & 15) of each 16-row block, k = 32*ks + 8*(l>>4) .. +7 ----
    const float* X = (const float*)p.A;
    u32x4 af[RB][NKS];
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
                    const float2 t = *(const float2*)(row + (in ? k0 + e : 0));
                    v[e] = in ? t.x : 0.f;
                    v[e + 1] = in ? t.y : 0.f;
                }
                af[rb][ks] = pack8<CT>(v);
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
                    const int tap = in ? (int)(((float)k + 0.5f) * inv_lda) : 0;
                    const int c = in ? k - tap * p.lda : 0;
                    int fr = f0 + tap;
                    fr = fr < 0 ? 0 : (fr >= len ? len - 1 : fr);
                    const int64_t gf = off + fr;
                    const float* src = c < g.f2 ? g.kps + gf * g.f2 + c : g.cams + gf * 12 + (c - g.f2);
                    const float2 tv = *(const float2*)src;
                    v[e] = in ? tv.x : 0.f;
                    v[e + 1] = in ? tv.y : 0.f;
                }
                af[rb][ks] = pack8<CT>(v);
            }
        }
    }

    const int nchunks = p.N / kExpChunkN;
    wload(0);
    wstore(0);
    if (nchunks > 1) wload(1);
    __syncthreads();

    const int frag_off = (lane & 15) * 4 + (((lane >> 4) + 2 * (((lane & 15) >> 2) & 3)) & 3);
    CT* Y = (CT*)p.Y;
    for (int ch = 0; ch < nchunks; ++ch) {
        const int buf = ch & 1;
        f32x4 acc[RB][4];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[rb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            u32x4 wf[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) wf[j] = wbuf[buf][ks * SLAB + j * 64 + frag_off];
#pragma unroll
            for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[rb][j] = mfma16<CT>(wf[j], af[rb][ks], acc[rb][j]);
        }
        // chunk ch+1 was loaded into registers during chunk ch-1; its LDS buffer was
        // last read in chunk ch-1, which every wave finished before the barrier below
        if (ch + 1 < nchunks) wstore(buf ^ 1);
        if (ch + 2 < nchunks) wload(ch + 2);

        // epilogue: lane holds channels n0 + 16j + 4(l>>4) + r of row rb*16 + (l & 15)
        const int n0 = ch * kExpChunkN;
        u32x4* stage = s_out[wid];
        typedef CT ct4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int nl = j * 16 + (lane >> 4) * 4;  // channel within the chunk
            const f32x4 sc = *(const f32x4*)&s_scale[n0 + nl];
            const f32x4 sh = *(const f32x4*)&s_shift[n0 + nl];
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) {
                ct4 o;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = __fadd_rn(__fmul_rn(acc[rb][j][r], sc[r]), sh[r]);
                    if (p.relu) v = v > 0.f ? v : 0.f;
                    o[r] = (CT)v;
                }
                const int row = rb * 16 + (lane & 15);
                const int c16 = nl >> 3;  // 16-byte chunk (8 channels), half (nl >> 2) & 1
                // the half is swapped on rows 8-15 of each 16: the 16 lanes of a write group
                // then cover all 32 banks (rows r and r + 8 otherwise shared them)
                char* dst = (char*)stage + row * 128 + ((c16 ^ (row & 7)) << 4) +
                            ((((nl >> 2) & 1) ^ ((row >> 3) & 1)) << 3);
                *(ct4*)dst = o;
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
            if (m < p.M) {
                u32x4* dst = (u32x4*)(Y + (int64_t)m * p.ldy + n0 + c16 * 8);
                if constexpr (NT)
                    __builtin_nontemporal_store(v, dst);
                else
                    *dst = v;
            }
        }
        asm volatile("" ::: "memory");
        __syncthreads();
    }
}

template <typename CT, int RB, bool GATHER, bool NT>
hipError_t launch_rb_nt(const ConvGemmParams& p, const GatherSrc& g, int nks, hipStream_t s) {
    const dim3 grid((p.M + 64 * RB - 1) / (64 * RB));
    switch (nks) {
        case 1: hipLaunchKernelGGL((expand_gemm_h16<CT, 1, RB, GATHER, NT>), grid, dim3(256), 0, s, p, g); break;
        case 2: hipLaunchKernelGGL((expand_gemm_h16<CT, 2, RB, GATHER, NT>), grid, dim3(256), 0, s, p, g); break;
        case 3: hipLaunchKernelGGL((expand_gemm_h16<CT, 3, RB, GATHER, NT>), grid, dim3(256), 0, s, p, g); break;
        case 4: hipLaunchKernelGGL((expand_gemm_h16<CT, 4, RB, GATHER, NT>), grid, dim3(256), 0, s, p, g); break;
        case 5: hipLaunchKernelGGL((expand_gemm_h16<CT, 5, RB, GATHER, NT>), grid, dim3(256), 0, s, p, g); break;
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
// Row blocks of 16 per wave: fewer rows per wave, fewer VGPRs and less LDS per
// workgroup, more resident waves to hide store / input latency, but the weight sweep is
// repeated for every workgroup.  4 where that instantiation still holds 2 waves per SIMD
// (<= 256 VGPR + AGPR: the plain loader with K <= 128 — 250), else 2 (the gathered
// loader's address arithmetic, or K up to 160, put RB = 4 at 280-327 registers = 1 wave
// per SIMD).  Measured at B = 8192 (round 1): plain K = 102: RB 4 -> 0.370, 2 -> 0.406,
// 1 -> 0.442 ms; gathered K = 138 (config 3): 4 -> 0.548, 3 -> 0.557, 2 -> 0.400 ms.
template <typename CT, bool GATHER>
hipError_t launch_t(const ConvGemmParams& p, const GatherSrc& g, int nks, hipStream_t s) {
    const bool nt = (int64_t)p.M * p.ldy * 2 > (int64_t)256 << 20;
    if (!GATHER && nks <= 4)
        return nt ? launch_rb_nt<CT, 4, GATHER, true>(p, g, nks, s) : launch_rb_nt<CT, 4, GATHER, false>(p, g, nks, s);
    return nt ? launch_rb_nt<CT, 2, GATHER, true>(p, g, nks, s) : launch_rb_nt<CT, 2, GATHER, false>(p, g, nks, s);
}

}  // namespace

bool expand_gemm_eligible(const ConvGemmParams& p, Act out_type, Act compute) {
    if (compute == Act::F32 || out_type != compute) return false;
    if (p.Ktap != p.K || p.dil != 1) return false;  // taps collapsed into one contiguous K run
    const int nks = (p.K + 31) / 32;
    if (nks < 1 || nks > 5 || nks * 32 > p.Kp) return false;  // K <= 160 (LDS for 2 WG/CU)
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
    const int nks = (p.K + 31) / 32;
    const GatherSrc none{};
    return compute == Act::BF16 ? launch_t<bf16, false>(p, none, nks, stream)
                                : launch_t<f16, false>(p, none, nks, stream);
}

hipError_t launch_expand_gemm_gather(const ConvGemmParams& p, const GatherSrc& g, Act compute,
                                     hipStream_t stream) {
    const int nks = (p.K + 31) / 32;
    return compute == Act::BF16 ? launch_t<bf16, true>(p, g, nks, stream) : launch_t<f16, true>(p, g, nks, stream);
}

}  // namespace vp3d
