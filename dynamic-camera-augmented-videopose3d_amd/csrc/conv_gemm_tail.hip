// Split-K tail of a split-fp16 (f16x3) conv-GEMM launch: the rows past a layer's last whole
// round of 256 x 256 tiles, spread over every CU.
//
// Why: sequence mode (the dilated TemporalModel over one long sequence, run.py --evaluate:
// TemporalModel.py:126-138, run.py:697-711) gives every block layer 65,536 + c rows (c = 2, 6,
// 18, 54, 162 ... the receptive-field halo of the layers after it), i.e. 4 whole rounds of
// 256 x 256 tiles plus ONE M-tile of 4 tiles.  conv_gemm_a4 ran that tail as 16 quarter-N tiles
// of 256 x 64 on 16 CUs, each a full-K chain: 45-78 us per k3 launch (block-4 k3, which has no
// tail, takes 0.807 ms for the 4 rounds; block-3 k3 0.885).  Here the tail's K range is cut into
// S slices as well: (N / 64) x S x (tail M-tiles) workgroups -- 256 for one M-tile -- each
// computing a 256 x 64 block over Kp / S and storing its f32 partial sums; a second launch adds
// the S partials in slice order per output and applies the epilogue of conv_gemm_a4's split
// path (BN in two roundings, ReLU, residual hi + lo, f16 hi / lo split or f32 rows, the range
// guard).  Deterministic from run to run, not the whole tile's bits (S chains instead of one:
// within 1e-6 relative, tests/test_gpu_lifter.py).
//
// Operands as conv_gemm_a4<_Float16, X3>: rows of f16 halves, each 32-wide K group [hi(32) |
// lo(32)] (A: activation rows, W: Layer::wx3); per 64-half K-step and accumulator the products
// W_hi.A_hi, W_hi.A_lo, W_lo.A_hi (the lo.lo term, 2^-22 relative, dropped), as a4 / q64.
// Operands staged through LDS as whole 128-byte lines, one K-step ahead.
#include "gemm_common.h"

namespace vp3d {
namespace {

using namespace gemm;

constexpr int TM = 256;  // rows per workgroup (4 waves x 64)
constexpr int TN = 64;   // channels per workgroup
constexpr int KS = 64;   // halves per K-step (one [hi | lo] group of 32 K values)

// part[slice][row - m_begin][n] (f32), rows_pad = tail M-tiles x 256.  X3: split-fp16 rows
// (CT = f16, 3 products per 32-wide K group); otherwise 16-bit rows (bf16 / fp16), a K-step's
// two 32-deep halves as two MFMAs (a4's k order within the tile).
// Per K-step the workgroup stages A (256 rows x 128 B) and W (64 rows x 128 B) in LDS -- 8
// consecutive lanes per 128-byte row, so every global load is whole lines -- double-buffered
// through registers (the next step's 10 loads per lane in flight under this step's MFMAs); the
// 16-byte chunk c of LDS row r sits at c ^ (r & 7), so a fragment read (16 rows, one chunk) is
// spread over the banks.  (Round 6, first form: fragments straight from global memory, 16
// rows per load instruction: 44-48 us per k3 tail, 21 us per 1x1 tail.)
// RBW: row blocks of 16 per wave (4: 256 rows per workgroup; 1: 64 rows, the f16x3 shrink of small
// batches -- 4x the workgroups, the same per-output chains)
template <typename CT, bool X3, int RBW = 4>
__global__ __launch_bounds__(256) void tail_split_kernel(ConvGemmParams p, int m_begin, int rows_pad,
                                                         int steps_per_unit, float* __restrict__ part) {
    constexpr int TMR = 64 * RBW;  // rows per workgroup
    constexpr int NA = TMR / 32;   // A rows staged per thread and K-step
    __shared__ __attribute__((aligned(16))) char smem[2][(TMR + TN) * 128];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wv = tid >> 6;
    const int g = lane >> 4;  // k chunk (8 elements) of this lane in a 32-deep half
    const int n0 = blockIdx.x * TN;
    const int slice = blockIdx.y;
    const int mt0 = blockIdx.z * TMR;  // the workgroup's first row (tail-relative)
    const int s0 = slice * steps_per_unit;

    // staging: this thread's NA A rows (tid / 8 + 32 i) and 2 W rows (tid / 8 + 32 i), chunk tid % 8
    const int sc = tid & 7;
    const int sr = tid >> 3;
    const CT* const A = (const CT*)p.A;
    const CT* const W = (const CT*)p.W;
    int srow[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        int m = m_begin + mt0 + sr + 32 * i;
        m = m < p.M ? m : p.M - 1;  // rows past M read a valid row; never stored
        srow[i] = src_row(p, m);
    }
    u32x4 st[NA + 2];
    auto gload = [&](int s) __attribute__((always_inline)) {
        const int k0 = s * KS;
        const int tap = k0 / p.Ktap;
        const int koff = k0 - tap * p.Ktap + 8 * sc;
#pragma unroll
        for (int i = 0; i < NA; ++i) st[i] = *(const u32x4*)(A + (int64_t)(srow[i] + tap * p.dil) * p.lda + koff);
#pragma unroll
        for (int i = 0; i < 2; ++i) st[NA + i] = *(const u32x4*)(W + (size_t)(n0 + sr + 32 * i) * p.Kp + k0 + 8 * sc);
    };
    auto lstore = [&](char* buf) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NA + 2; ++i) {
            const int r = i < NA ? sr + 32 * i : TMR + sr + 32 * (i - NA);
            *(u32x4*)(buf + r * 128 + ((sc ^ (r & 7)) << 4)) = st[i];
        }
    };
    // fragment of LDS row r, logical chunk c
    auto frag = [&](const char* buf, int r, int c) __attribute__((always_inline)) -> u32x4 {
        return *(const u32x4*)(buf + r * 128 + ((c ^ (r & 7)) << 4));
    };
    f32x4 acc[RBW][4];
#pragma unroll
    for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[rb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    gload(s0);
    lstore(smem[0]);
    __syncthreads();
    const int fr = lane & 15;
    for (int i = 0; i < steps_per_unit; ++i) {
        const char* buf = smem[i & 1];
        if (i + 1 < steps_per_unit) gload(s0 + i + 1);
        u32x4 fa[RBW][2], fw[4][2];
#pragma unroll
        for (int rb = 0; rb < RBW; ++rb) {
            fa[rb][0] = frag(buf, 16 * RBW * wv + 16 * rb + fr, g);
            fa[rb][1] = frag(buf, 16 * RBW * wv + 16 * rb + fr, 4 + g);
        }
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
            fw[cb][0] = frag(buf, TMR + 16 * cb + fr, g);
            fw[cb][1] = frag(buf, TMR + 16 * cb + fr, 4 + g);
        }
        // transposed issue (W as the MFMA's A operand): a lane's 4 results are 4 consecutive
        // channels of one row -- one 16-byte store each.  Per accumulator: hh, hl, lh (X3).
#pragma unroll
        for (int rb = 0; rb < RBW; ++rb)
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) {
                if constexpr (X3) {
                    acc[rb][cb] = mfma16<CT>(fw[cb][0], fa[rb][0], acc[rb][cb]);
                    acc[rb][cb] = mfma16<CT>(fw[cb][0], fa[rb][1], acc[rb][cb]);
                    acc[rb][cb] = mfma16<CT>(fw[cb][1], fa[rb][0], acc[rb][cb]);
                } else {
                    acc[rb][cb] = mfma16<CT>(fw[cb][0], fa[rb][0], acc[rb][cb]);
                    acc[rb][cb] = mfma16<CT>(fw[cb][1], fa[rb][1], acc[rb][cb]);
                }
            }
        if (i + 1 < steps_per_unit) {
            lstore(smem[(i + 1) & 1]);  // the buffer read one step ago (a barrier since)
            __syncthreads();
        }
    }
    // lane l of block (rb, cb): channels n0 + 16 cb + 4 g + 0..3 of row 16 RBW wv + 16 rb + (l & 15)
    float* const pbase = part + (size_t)slice * rows_pad * p.N;
#pragma unroll
    for (int rb = 0; rb < RBW; ++rb) {
        const int mloc = mt0 + 16 * RBW * wv + 16 * rb + fr;
        if (m_begin + mloc >= p.M) continue;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
            *(f32x4*)(pbase + (size_t)mloc * p.N + n0 + 16 * cb + 4 * g) = acc[rb][cb];
    }
}

// one thread per (row, 8 channels): the S partials summed in slice order, then a4's split
// epilogue (gemm::epilogue_tp_x3's arithmetic)
template <bool OUT_F32, bool HAS_R>
__global__ __launch_bounds__(256) void tail_reduce_x3_kernel(ConvGemmParams p, int m_begin, int rows, int rows_pad,
                                                             int S, const float* __restrict__ part) {
    const int per_row = p.N / 8;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)rows * per_row) return;
    const int mloc = (int)(t / per_row);
    const int c8 = (int)(t - (int64_t)mloc * per_row) * 8;
    const float* pp = part + (size_t)mloc * p.N + c8;
    const size_t plane = (size_t)rows_pad * p.N;
    f32x4 v0 = *(const f32x4*)pp, v1 = *(const f32x4*)(pp + 4);
    for (int q = 1; q < S; ++q) {
        v0 = v0 + *(const f32x4*)(pp + q * plane);
        v1 = v1 + *(const f32x4*)(pp + q * plane + 4);
    }
    float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    const f32x4 sc0 = *(const f32x4*)(p.scale + c8), sc1 = *(const f32x4*)(p.scale + c8 + 4);
    const f32x4 sh0 = *(const f32x4*)(p.shift + c8), sh1 = *(const f32x4*)(p.shift + c8 + 4);
    const float sc[8] = {sc0[0], sc0[1], sc0[2], sc0[3], sc1[0], sc1[1], sc1[2], sc1[3]};
    const float sh[8] = {sh0[0], sh0[1], sh0[2], sh0[3], sh1[0], sh1[1], sh1[2], sh1[3]};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        float x = __fadd_rn(__fmul_rn(v[e], sc[e]), sh[e]);
        if (p.relu) x = __builtin_bit_cast(float, max(__builtin_bit_cast(int, x), 0));  // ReLU, -0 -> +0
        v[e] = x;
    }
    const int m = m_begin + mloc;
    // channel n's halves sit at 64 (n / 32) + n % 32 (hi) and + 32 (lo) of a split row
    const int hoff = 64 * (c8 / 32) + (c8 % 32);
    if constexpr (HAS_R) {
        const f16* rp = (const f16*)p.R + (int64_t)res_row(p, m) * p.ldr + hoff;
        const u32x4 rh = *(const u32x4*)rp, rl = *(const u32x4*)(rp + 32);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float t0, t1;
            x3_res_sum2(rh[e], rl[e], t0, t1);
            v[2 * e] += t0;
            v[2 * e + 1] += t1;
        }
    }
    if constexpr (OUT_F32) {
        float* y = (float*)p.Y + (int64_t)m * p.ldy + c8;
        *(f32x4*)y = f32x4{v[0], v[1], v[2], v[3]};
        *(f32x4*)(y + 4) = f32x4{v[4], v[5], v[6], v[7]};
    } else {
        u32x4 oh, ol;
        float vmax = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            oh[e] = x3_hi2(v[2 * e], v[2 * e + 1]);
            ol[e] = x3_split_lo2(oh[e], v[2 * e], v[2 * e + 1]);
            vmax = x3_absmax2(vmax, v[2 * e], v[2 * e + 1]);
        }
        f16* y = (f16*)p.Y + (int64_t)m * p.ldy + hoff;
        *(u32x4*)y = oh;
        *(u32x4*)(y + 32) = ol;
        x3_range_flag(vmax, p.scale, p.N);
    }
}

// the 16-bit reduce: bf16 / fp16 rows out, a4's packed epilogue arithmetic (BN in two
// roundings; with a residual ReLU then + r in f32, one rounding to CT; without one the ReLU
// before the rounding -- the same bits as a4's max on the rounded pair)
template <typename CT, bool HAS_R>
__global__ __launch_bounds__(256) void tail_reduce16_kernel(ConvGemmParams p, int m_begin, int rows, int rows_pad,
                                                            int S, const float* __restrict__ part) {
    const int per_row = p.N / 8;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)rows * per_row) return;
    const int mloc = (int)(t / per_row);
    const int c8 = (int)(t - (int64_t)mloc * per_row) * 8;
    const float* pp = part + (size_t)mloc * p.N + c8;
    const size_t plane = (size_t)rows_pad * p.N;
    f32x4 v0 = *(const f32x4*)pp, v1 = *(const f32x4*)(pp + 4);
    for (int q = 1; q < S; ++q) {
        v0 = v0 + *(const f32x4*)(pp + q * plane);
        v1 = v1 + *(const f32x4*)(pp + q * plane + 4);
    }
    const float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    const int m = m_begin + mloc;
    typename Pack8<CT>::type r8;
    if constexpr (HAS_R)
        r8 = __builtin_bit_cast(typename Pack8<CT>::type, *(const u32x4*)((const CT*)p.R + (int64_t)res_row(p, m) * p.ldr + c8));
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        float x = __fadd_rn(__fmul_rn(v[e], p.scale[c8 + e]), p.shift[c8 + e]);
        x = __builtin_bit_cast(float, max(__builtin_bit_cast(int, x), 0));  // ReLU (a4: relu == 1), -0 -> +0
        if constexpr (HAS_R) x = x + (float)r8[e];
        o[e] = x;
    }
    *(u32x4*)((CT*)p.Y + (int64_t)m * p.ldy + c8) = pack8<CT>(o);
}

// the shrink's reduce: one thread per (row, real channel n < N_out): the S partials in slice
// order, then scale / shift (two roundings, no ReLU), f32 into the pose rows
__global__ __launch_bounds__(256) void shrink_reduce_x3_kernel(ConvGemmParams p, int n_out, int m_begin, int rows,
                                                               int rows_pad, int S, const float* __restrict__ part) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)rows * n_out) return;
    const int mloc = (int)(t / n_out);
    const int n = (int)(t - (int64_t)mloc * n_out);
    const float* pp = part + (size_t)mloc * TN + n;
    float v = pp[0];
    for (int q = 1; q < S; ++q) v += pp[(size_t)q * rows_pad * TN];
    ((float*)p.Y)[(int64_t)(m_begin + mloc) * p.ldy + n] = __fadd_rn(__fmul_rn(v, p.scale[n]), p.shift[n]);
}

}  // namespace

// S for a tail of `rows` rows: about one workgroup per CU, S | Kp / 64, the partials within
// the split workspace; 0 when the shape does not fit this path
static int tail_slices(const ConvGemmParams& p, int rows, int ncu) {
    if (rows <= 0 || p.N % TN != 0 || p.Kp % KS != 0 || p.Ktap % KS != 0 || p.lda % 8 != 0 || p.ldy % 8 != 0 ||
        (p.R && p.ldr % 8 != 0))
        return 0;
    const int mt = (rows + TM - 1) / TM;
    const int nsteps = p.Kp / KS;
    const size_t plane = (size_t)mt * TM * p.N * sizeof(float);
    int S = ncu / ((p.N / TN) * mt);
    if (S > nsteps) S = nsteps;
    while (S > 1 && (nsteps % S != 0 || (size_t)S * plane > kSplitPartBytes)) --S;
    return S >= 2 ? S : 0;
}

bool conv_gemm_tail_fits(const ConvGemmParams& p, int m_begin, int ncu, bool need_ws) {
    return (!need_ws || p.sk_part != nullptr) && tail_slices(p, p.M - m_begin, ncu) > 0;
}

hipError_t launch_conv_gemm_tail16(const ConvGemmParams& p, int m_begin, Act compute, int ncu, hipStream_t stream) {
    const int rows = p.M - m_begin;
    const int S = tail_slices(p, rows, ncu);
    if (S == 0 || !p.sk_part || p.relu != 1) return hipErrorInvalidValue;
    const int mt = (rows + TM - 1) / TM;
    const int rows_pad = mt * TM;
    const dim3 g(p.N / TN, S, mt);
    const int spu = (p.Kp / KS) / S;
    const unsigned blocks = (unsigned)(((int64_t)rows * (p.N / 8) + 255) / 256);
    const float* part = p.sk_part;
    if (compute == Act::BF16) {
        hipLaunchKernelGGL((tail_split_kernel<bf16, false>), g, dim3(256), 0, stream, p, m_begin, rows_pad, spu, p.sk_part);
        if (p.R)
            hipLaunchKernelGGL((tail_reduce16_kernel<bf16, true>), dim3(blocks), dim3(256), 0, stream, p, m_begin, rows,
                               rows_pad, S, part);
        else
            hipLaunchKernelGGL((tail_reduce16_kernel<bf16, false>), dim3(blocks), dim3(256), 0, stream, p, m_begin, rows,
                               rows_pad, S, part);
    } else {
        hipLaunchKernelGGL((tail_split_kernel<f16, false>), g, dim3(256), 0, stream, p, m_begin, rows_pad, spu, p.sk_part);
        if (p.R)
            hipLaunchKernelGGL((tail_reduce16_kernel<f16, true>), dim3(blocks), dim3(256), 0, stream, p, m_begin, rows,
                               rows_pad, S, part);
        else
            hipLaunchKernelGGL((tail_reduce16_kernel<f16, false>), dim3(blocks), dim3(256), 0, stream, p, m_begin, rows,
                               rows_pad, S, part);
    }
    return hipGetLastError();
}

hipError_t launch_conv_gemm_tail_x3(const ConvGemmParams& p, int m_begin, bool out_f32, int ncu, hipStream_t stream) {
    const int rows = p.M - m_begin;
    const int S = tail_slices(p, rows, ncu);
    if (S == 0 || !p.sk_part) return hipErrorInvalidValue;
    const int mt = (rows + TM - 1) / TM;
    const int rows_pad = mt * TM;
    hipLaunchKernelGGL((tail_split_kernel<f16, true>), dim3(p.N / TN, S, mt), dim3(256), 0, stream, p, m_begin,
                       rows_pad, (p.Kp / KS) / S, p.sk_part);
    const unsigned blocks = (unsigned)(((int64_t)rows * (p.N / 8) + 255) / 256);
    const bool has_r = p.R != nullptr;
    if (out_f32) {
        if (has_r)
            hipLaunchKernelGGL((tail_reduce_x3_kernel<true, true>), dim3(blocks), dim3(256), 0, stream, p, m_begin,
                               rows, rows_pad, S, (const float*)p.sk_part);
        else
            hipLaunchKernelGGL((tail_reduce_x3_kernel<true, false>), dim3(blocks), dim3(256), 0, stream, p, m_begin,
                               rows, rows_pad, S, (const float*)p.sk_part);
    } else {
        if (has_r)
            hipLaunchKernelGGL((tail_reduce_x3_kernel<false, true>), dim3(blocks), dim3(256), 0, stream, p, m_begin,
                               rows, rows_pad, S, (const float*)p.sk_part);
        else
            hipLaunchKernelGGL((tail_reduce_x3_kernel<false, false>), dim3(blocks), dim3(256), 0, stream, p, m_begin,
                               rows, rows_pad, S, (const float*)p.sk_part);
    }
    return hipGetLastError();
}

}  // namespace vp3d

namespace vp3d {
// the f16x3 shrink: p.N = the real output channels (<= 64), p.W = the shrink's split weights
// (zero rows past N), p.scale = its scale_x3 (padded to 64); rows in chunks whose 2 K-slices of
// 64-column partials fit the split workspace
hipError_t launch_conv_gemm_x3_shrink(const ConvGemmParams& p_in, hipStream_t stream) {
    constexpr int S = 2;
    const int n_out = p_in.N;
    if (n_out > TN || !p_in.sk_part || p_in.Kp % (KS * S) != 0 || p_in.Ktap % KS != 0 || p_in.lda % 8 != 0)
        return hipErrorInvalidValue;
    ConvGemmParams p = p_in;
    p.N = TN;
    const int chunk = (int)(kSplitPartBytes / ((size_t)S * TN * sizeof(float)) / TM * TM);
    // below 32,768 rows 64-row workgroups (4x as many: 8,192 windows 0.026 ms vs 0.036 on the narrow
    // exact-f32 kernel, profiles/r06_x3_small_shrink_ab.txt), the
    // same per-output chains (bit-identical across batch sizes, test_config4_eight_shards_bit_equal)
    const bool small = p_in.M < 32768;
    for (int m0 = 0; m0 < p_in.M; m0 += chunk) {
        const int m1 = m0 + chunk < p_in.M ? m0 + chunk : p_in.M;
        p.M = m1;  // the row bound of this chunk (rows past it clamp and are not stored)
        const int rows = m1 - m0;
        const int tmr = small ? 64 : TM;
        const int mt = (rows + tmr - 1) / tmr;
        if (small)
            hipLaunchKernelGGL((tail_split_kernel<f16, true, 1>), dim3(1, S, mt), dim3(256), 0, stream, p, m0, mt * tmr,
                               (p.Kp / KS) / S, p.sk_part);
        else
            hipLaunchKernelGGL((tail_split_kernel<f16, true, 4>), dim3(1, S, mt), dim3(256), 0, stream, p, m0, mt * tmr,
                               (p.Kp / KS) / S, p.sk_part);
        const unsigned blocks = (unsigned)(((int64_t)rows * n_out + 255) / 256);
        hipLaunchKernelGGL(shrink_reduce_x3_kernel, dim3(blocks), dim3(256), 0, stream, p, n_out, m0, rows, mt * tmr, S,
                           (const float*)p.sk_part);
    }
    return hipGetLastError();
}
}  // namespace vp3d
