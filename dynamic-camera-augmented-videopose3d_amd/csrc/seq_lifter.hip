// Kernels of the fork's other trajectory-conditioned lifters in eval mode
// (SURVEY.md §8(f) rank 4): CoupledTransformer (reference CamTransformer.py:95-205)
// and CoupledLSTM (CamLSTM.py:47-129), batched over windows or over the sliding
// windows of one sequence (sliding_window, CamTransformer.py:72-92).  The Linear
// layers run on the f32 conv-GEMM (conv_gemm.hip); these are the rest:
//
//   concat_frames_kernel    [flat 2D | flat K.E] rows (CamTransformer.py:187-190)
//   pe_layernorm_kernel     LayerNorm(P[frame(w, t)] + pe[t]) per window row: the input
//                           projection P is computed once per frame and shared by every
//                           window that contains the frame (:193-195)
//   layernorm_kernel        the post-norm LayerNorms of nn.TransformerEncoderLayer
//   attention_mfma_kernel   softmax(q k^T / sqrt(dh)) v per (window, head) on the f32 MFMA
//                           (full layers)
//   attention_last_kernel   the same for the last query only: the last encoder layer only
//                           needs it (CamTransformer.py:201 keeps enc_out[:, -1])
//   attention_kernel        scalar fallback (head dims without an MFMA variant)
//   lstm_kernel             the stacked nn.LSTM recurrence (gate order i, f, g, o; zero
//                           initial state) of a tile of windows, persistent over all time
//                           steps; layer 0's input projection is precomputed per frame
//
// f32 throughout (the reference evaluates these models in f32).
#include <algorithm>
#include <climits>

#include "kernels.h"

#pragma clang fp contract(off)

namespace vp3d {
namespace {

__device__ __forceinline__ float wave_sum(float v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ void concat_frames_kernel(const float* __restrict__ a, int fa, const float* __restrict__ b, int fb,
                                     int64_t rows, float* __restrict__ out) {
    const int w = fa + fb;
    const int64_t total = rows * w;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = e / w;
        const int c = (int)(e - r * w);
        out[e] = c < fa ? a[r * fa + c] : b[r * fb + (c - fa)];
    }
}

// One wave per output row m = (w, t): x = X[w * win_stride + t] (+ pe[t]); LayerNorm
// over d (biased variance, eps), as ATen: y = (x - mean) * rstd * gamma + beta.
__global__ __launch_bounds__(256) void layernorm_rows_kernel(const float* __restrict__ X, int d, int64_t n_rows,
                                                             int W, int win_stride, const float* __restrict__ pe,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, float eps,
                                                             float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (m >= n_rows) return;
    const int64_t w = m / W;
    const int t = (int)(m - w * W);
    const float* x = X + (w * win_stride + t) * (int64_t)d;
    float v[16];  // d <= 1024
    const int per = (d + 63) / 64;
    float s = 0.f;
    for (int i = 0; i < per; ++i) {
        const int c = lane + 64 * i;
        float xv = 0.f;
        if (c < d) {
            xv = x[c];
            if (pe) xv = xv + pe[(int64_t)t * d + c];
        }
        v[i] = xv;
        s += xv;
    }
    const float mean = wave_sum(s) / (float)d;
    float q = 0.f;
    for (int i = 0; i < per; ++i) {
        const int c = lane + 64 * i;
        const float dv = c < d ? v[i] - mean : 0.f;
        q += dv * dv;
    }
    const float var = wave_sum(q) / (float)d;
    const float rstd = 1.0f / sqrtf(var + eps);
    float* o = out + m * d;
    for (int i = 0; i < per; ++i) {
        const int c = lane + 64 * i;
        if (c < d) o[c] = (v[i] - mean) * rstd * gamma[c] + beta[c];
    }
}

// The same LayerNorm for d % 4 == 0, d <= 256: LPR = d/4 lanes per row (a power of two),
// one float4 per lane, 64/LPR rows per wave-instruction and U such row groups in flight
// per wave (grid-stride over row groups).  The one-wave-per-row kernel above spent most
// of its time waiting on one 512-B row per wave (≈2.4 TB/s at d = 128); with 8 rows of
// independent 16-B loads in flight per wave this one streams the rows.
template <int LPR, int U>
__global__ __launch_bounds__(256) void layernorm_rows_vec_kernel(const float* __restrict__ X, int d, int64_t n_rows,
                                                                 int W, int win_stride,
                                                                 const float* __restrict__ pe,
                                                                 const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta, float eps,
                                                                 float* __restrict__ out) {
    constexpr int RPI = 64 / LPR;  // rows per wave-instruction
    const int lane = threadIdx.x & 63;
    const int sub = lane / LPR, c4 = lane % LPR;
    const bool cv = c4 * 4 < d;
    const float4 g = cv ? *(const float4*)(gamma + c4 * 4) : float4{0.f, 0.f, 0.f, 0.f};
    const float4 bb = cv ? *(const float4*)(beta + c4 * 4) : float4{0.f, 0.f, 0.f, 0.f};
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t n_waves = (int64_t)gridDim.x * 4;
    for (int64_t base = wave * (RPI * U); base < n_rows; base += n_waves * (RPI * U)) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t m = base + u * RPI + sub;
            v[u] = float4{0.f, 0.f, 0.f, 0.f};
            if (m < n_rows && cv) {
                const int64_t w = n_rows < INT32_MAX ? (int64_t)((uint32_t)m / (uint32_t)W) : m / W;
                const int t = (int)(m - w * W);
                v[u] = *(const float4*)(X + (w * win_stride + t) * (int64_t)d + c4 * 4);
                if (pe) {
                    const float4 p = *(const float4*)(pe + (int64_t)t * d + c4 * 4);
                    v[u].x = v[u].x + p.x;
                    v[u].y = v[u].y + p.y;
                    v[u].z = v[u].z + p.z;
                    v[u].w = v[u].w + p.w;
                }
            }
        }
        float mean[U], rstd[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float s = (v[u].x + v[u].y) + (v[u].z + v[u].w);
#pragma unroll
            for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
            mean[u] = s / (float)d;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float a = cv ? v[u].x - mean[u] : 0.f, b = cv ? v[u].y - mean[u] : 0.f;
            const float c = cv ? v[u].z - mean[u] : 0.f, e = cv ? v[u].w - mean[u] : 0.f;
            float q = (a * a + b * b) + (c * c + e * e);
#pragma unroll
            for (int o = LPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
            rstd[u] = 1.0f / sqrtf(q / (float)d + eps);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t m = base + u * RPI + sub;
            if (m < n_rows && cv) {
                float4 o;
                o.x = (v[u].x - mean[u]) * rstd[u] * g.x + bb.x;
                o.y = (v[u].y - mean[u]) * rstd[u] * g.y + bb.y;
                o.z = (v[u].z - mean[u]) * rstd[u] * g.z + bb.z;
                o.w = (v[u].w - mean[u]) * rstd[u] * g.w + bb.w;
                *(float4*)(out + m * d + c4 * 4) = o;
            }
        }
    }
}

// Multi-head self-attention of one window and one head; QKV rows of 3d floats
// ([q | k | v], head h at columns h*DH), output O rows of d floats.
template <int DH>
__global__ __launch_bounds__(256) void attention_kernel(const float* __restrict__ QKV, int W, int d, int last_only,
                                                        float scale, float* __restrict__ O) {
    extern __shared__ float sm[];
    float* Ks = sm;            // [W][DH]
    float* Vs = sm + W * DH;   // [W][DH]
    const int w = blockIdx.x, h = blockIdx.y;
    const int64_t row0 = (int64_t)w * W;
    const int ld = 3 * d;
    for (int e = threadIdx.x; e < W * DH; e += blockDim.x) {
        const int j = e / DH, c = e - j * DH;
        const float* r = QKV + (row0 + j) * ld + h * DH + c;
        Ks[e] = r[d];
        Vs[e] = r[2 * d];
    }
    __syncthreads();
    const int t_begin = last_only ? W - 1 : 0;
    for (int t = t_begin + (int)threadIdx.x; t < W; t += blockDim.x) {
        float q[DH], o[DH];
        const float* qr = QKV + (row0 + t) * ld + h * DH;
#pragma unroll
        for (int c = 0; c < DH; ++c) {
            q[c] = qr[c];
            o[c] = 0.f;
        }
        float mx = -INFINITY, l = 0.f;
        for (int j = 0; j < W; ++j) {
            float s = 0.f;
#pragma unroll
            for (int c = 0; c < DH; ++c) s = fmaf(q[c], Ks[j * DH + c], s);
            s = s * scale;
            if (s > mx) {
                const float corr = __expf(mx - s);
                l *= corr;
#pragma unroll
                for (int c = 0; c < DH; ++c) o[c] *= corr;
                mx = s;
            }
            const float pj = __expf(s - mx);
            l += pj;
#pragma unroll
            for (int c = 0; c < DH; ++c) o[c] = fmaf(pj, Vs[j * DH + c], o[c]);
        }
        const float inv = 1.0f / l;
        float* orow = O + (last_only ? (int64_t)w : row0 + t) * d + h * DH;
#pragma unroll
        for (int c = 0; c < DH; ++c) orow[c] = o[c] * inv;
    }
}

// Full self-attention of one (window, head) on the f32 MFMA (v_mfma_f32_16x16x4_f32):
// each wave takes 16-query tiles; S^T = K Q^T per 16-key block (keys down the
// accumulator rows, queries across lanes), softmax over the keys in registers plus two
// cross-lane-group shuffles, then O^T += V^T P^T where P^T is consumed straight from the
// S^T accumulators (the MFMA k-slot of lane group g, register r is key 4g + r of the
// block on both operands, so no transpose is needed).  K and V in LDS, row pitch 36
// floats (conflict-free for both access patterns).
constexpr int ATT_LD = 36;
constexpr int ATT_WMAX = 256;

template <int DH>
__global__ __launch_bounds__(256) void attention_mfma_kernel(const float* __restrict__ QKV, int W, int d,
                                                             float scale, float* __restrict__ O) {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    static_assert(DH == 16 || DH == 32, "head dim");
    __shared__ __attribute__((aligned(16))) float Ks[ATT_WMAX * ATT_LD];
    __shared__ __attribute__((aligned(16))) float Vs[ATT_WMAX * ATT_LD];
    const int w = blockIdx.x, h = blockIdx.y;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t row0 = (int64_t)w * W;
    const int ld = 3 * d;
    const int nkb = (W + 15) / 16;
    // K, V rows of the window as 16-byte pieces (d, DH multiples of 4: launch_attention)
    for (int e = threadIdx.x; e < nkb * 16 * (DH / 4); e += blockDim.x) {
        const int j = e / (DH / 4), c = (e - j * (DH / 4)) * 4;
        f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
        if (j < W) {
            const float* r = QKV + (row0 + j) * ld + h * DH + c;
            kv = *(const f32x4*)(r + d);
            vv = *(const f32x4*)(r + 2 * d);
        }
        // K columns permuted (c = 4s + g stored at g * DH/4 + s): the QK^T operand of lane
        // group g is then DH/4 consecutive floats, read with 16-byte LDS reads
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) Ks[j * ATT_LD + e2 * (DH / 4) + c / 4] = kv[e2];
        *(f32x4*)&Vs[j * ATT_LD + c] = vv;
    }
    __syncthreads();
    const int g = lane >> 4, lq = lane & 15;
    constexpr int NS = DH / 4;
    for (int qt = wid; qt < nkb; qt += 4) {
        const int q = qt * 16 + lq;
        float qf[NS];
        const float* qr = QKV + (row0 + (q < W ? q : W - 1)) * ld + h * DH;
#pragma unroll
        for (int s = 0; s < NS; ++s) qf[s] = qr[4 * s + g] * scale;
        f32x4 S[ATT_WMAX / 16];
        float mx = -INFINITY;
        // two key blocks per pass: two independent MFMA chains (rows past W of the last
        // block read zeroed LDS rows and are masked below)
#pragma unroll
        for (int kb = 0; kb < ATT_WMAX / 16; kb += 2) {
            if (kb < nkb) {
                f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
                const float* kr = Ks + (kb * 16 + lq) * ATT_LD + g * NS;
                f32x4 k0[NS / 4], k1[NS / 4];
#pragma unroll
                for (int u = 0; u < NS / 4; ++u) {
                    k0[u] = *(const f32x4*)(kr + 4 * u);
                    k1[u] = *(const f32x4*)(kr + 16 * ATT_LD + 4 * u);
                }
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(k0[s / 4][s % 4], qf[s], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(k1[s / 4][s % 4], qf[s], acc1, 0, 0, 0);
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (kb * 16 + 4 * g + r >= W) acc0[r] = -INFINITY;
                    if ((kb + 1) * 16 + 4 * g + r >= W) acc1[r] = -INFINITY;
                    mx = fmaxf(mx, acc0[r]);
                    mx = fmaxf(mx, acc1[r]);
                }
                S[kb] = acc0;
                S[kb + 1] = acc1;
            }
        }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        float l = 0.f;
#pragma unroll
        for (int kb = 0; kb < ATT_WMAX / 16; ++kb) {
            if (kb < nkb) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float p = __expf(S[kb][r] - mx);
                    S[kb][r] = p;
                    l += p;
                }
            }
        }
        l += __shfl_xor(l, 16, 64);
        l += __shfl_xor(l, 32, 64);
        // P.V with one accumulator per (r, ib): 4 * DH/16 independent MFMA chains instead
        // of DH/16 chains of 4 * nkb dependent MFMAs (the chain latency bounded the kernel)
        f32x4 o4[4][DH / 16];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int ib = 0; ib < DH / 16; ++ib) o4[r][ib] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < ATT_WMAX / 16; ++kb) {
            if (kb < nkb) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float* vr = Vs + (kb * 16 + 4 * g + r) * ATT_LD + lq;
#pragma unroll
                    for (int ib = 0; ib < DH / 16; ++ib)
                        o4[r][ib] = __builtin_amdgcn_mfma_f32_16x16x4f32(vr[ib * 16], S[kb][r], o4[r][ib], 0, 0, 0);
                }
            }
        }
        f32x4 o[DH / 16];
#pragma unroll
        for (int ib = 0; ib < DH / 16; ++ib) o[ib] = (o4[0][ib] + o4[1][ib]) + (o4[2][ib] + o4[3][ib]);
        // o[ib][r]: dim ib*16 + 4g + r of query qt*16 + lq
        if (q < W) {
            const float inv = 1.0f / l;
            float* orow = O + (row0 + q) * d + h * DH;
#pragma unroll
            for (int ib = 0; ib < DH / 16; ++ib) {
                f32x4 v = o[ib];
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = v[r] * inv;
                *(f32x4*)(orow + ib * 16 + 4 * g) = v;
            }
        }
    }
}

// Attention of the LAST query only (the last encoder layer: CamTransformer.py:201 keeps
// enc_out[:, -1]): one wave per (window, head), lanes over the keys; each lane streams its
// keys' K and V rows (DH contiguous floats) once, softmax by wave reductions, the 64
// per-lane partial outputs summed through LDS.  Bandwidth-bound on the K/V rows.
template <int DH>
__global__ __launch_bounds__(1024) void attention_last_kernel(const float* __restrict__ QKV, int W, int d,
                                                              float scale, float* __restrict__ O) {
    __shared__ float part[16][64][DH + 1];
    const int w = blockIdx.x;
    const int h = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t row0 = (int64_t)w * W;
    const int ld = 3 * d;
    float q[DH];
    const float* qr = QKV + (row0 + W - 1) * ld + h * DH;
#pragma unroll
    for (int c = 0; c < DH; ++c) q[c] = qr[c] * scale;
    constexpr int KPL = 4;  // keys per lane (W <= 256)
    float sc[KPL];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
        const int j = lane + 64 * i;
        float sv = -INFINITY;
        if (j < W) {
            const float* kr = QKV + (row0 + j) * ld + d + h * DH;
            float a = 0.f;
#pragma unroll
            for (int c = 0; c < DH; ++c) a = fmaf(q[c], kr[c], a);
            sv = a;
        }
        sc[i] = sv;
        mx = fmaxf(mx, sv);
    }
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    float l = 0.f;
    float acc[DH];
#pragma unroll
    for (int c = 0; c < DH; ++c) acc[c] = 0.f;
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
        const int j = lane + 64 * i;
        if (j < W) {
            const float p = __expf(sc[i] - mx);
            l += p;
            const float* vr = QKV + (row0 + j) * ld + 2 * d + h * DH;
#pragma unroll
            for (int c = 0; c < DH; ++c) acc[c] = fmaf(p, vr[c], acc[c]);
        }
    }
    for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o, 64);
#pragma unroll
    for (int c = 0; c < DH; ++c) part[h][lane][c] = acc[c];
    __syncthreads();
    if (lane < DH) {
        float sum = 0.f;
        for (int i = 0; i < 64; ++i) sum += part[h][i][lane];
        O[(int64_t)w * d + h * DH + lane] = sum / l;
    }
}

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// Stacked LSTM over W steps for a tile of NW windows.  Thread (u, half): hidden unit u
// (0..H-1) of windows [half*NWH, half*NWH + NWH); it owns that unit's four gates and
// cell state.  Weights are read transposed ([k][4H], coalesced across units) from L2 every
// step, once per tile: the tile width NW sets how often the whole recurrence re-reads them
// (NW = 32 for <= 2 layers, the run.py configuration: half the weight traffic of NW = 16,
// the hidden states of both layers in 64 KiB of LDS).  The previous hidden states of the
// tile live in LDS and are read 4 units at a time (ds_read_b128, broadcast across the
// wave); every gate sum still accumulates k in ascending order.
constexpr int LSTM_MAXL = 4;

template <int H, int NW, int MAXL>
__global__ __launch_bounds__(2 * H) void lstm_kernel(LstmParams p) {
    constexpr int NWH = NW / 2;
    __shared__ __attribute__((aligned(16))) float hs[MAXL][2][NW][H];  // [layer][buffer][window][unit]
    const int u = threadIdx.x % H;
    const int half = threadIdx.x / H;
    const int w0 = blockIdx.x * NW;
    for (int e = threadIdx.x; e < MAXL * 2 * NW * H; e += blockDim.x) (&hs[0][0][0][0])[e] = 0.f;
    float c[MAXL][NWH];
#pragma unroll
    for (int l = 0; l < MAXL; ++l)
#pragma unroll
        for (int i = 0; i < NWH; ++i) c[l][i] = 0.f;
    __syncthreads();
    const int G = 4 * H;
    int cur = 0;
    // acc[q][i] += sum_k h[i][k] * WT[k][q*H + u], k ascending
    auto gemv = [&](float (&acc)[4][NWH], const float* WT, const float* h) {
        for (int k = 0; k < H; k += 4) {
            float wv[4][4];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                for (int q = 0; q < 4; ++q) wv[kk][q] = WT[(k + kk) * G + q * H + u];
#pragma unroll
            for (int i = 0; i < NWH; ++i) {
                const float4 hv = *(const float4*)&h[i * H + k];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    acc[q][i] = fmaf(hv.x, wv[0][q], acc[q][i]);
                    acc[q][i] = fmaf(hv.y, wv[1][q], acc[q][i]);
                    acc[q][i] = fmaf(hv.z, wv[2][q], acc[q][i]);
                    acc[q][i] = fmaf(hv.w, wv[3][q], acc[q][i]);
                }
            }
        }
    };
    for (int t = 0; t < p.W; ++t) {
        for (int l = 0; l < p.L; ++l) {
            float acc[4][NWH];
            // layer input: precomputed projection (l = 0) or the new hidden state of layer l-1
#pragma unroll
            for (int i = 0; i < NWH; ++i) {
                const int w = w0 + half * NWH + i;
                if (l == 0) {
                    const float* g = p.gin + ((int64_t)(w < p.n_win ? w : 0) * p.win_stride + t) * G;
#pragma unroll
                    for (int q = 0; q < 4; ++q) acc[q][i] = g[q * H + u];
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) acc[q][i] = p.bias[l][q * H + u];
                }
            }
            if (l > 0) gemv(acc, p.wih_t[l], &hs[l - 1][cur ^ 1][half * NWH][0]);
            gemv(acc, p.whh_t[l], &hs[l][cur][half * NWH][0]);
#pragma unroll
            for (int i = 0; i < NWH; ++i) {
                const float ig = sigm(acc[0][i]), fg = sigm(acc[1][i]);
                const float gg = tanhf(acc[2][i]), og = sigm(acc[3][i]);
                float cc = c[0][0];
#pragma unroll
                for (int ll = 0; ll < MAXL; ++ll)
                    if (ll == l) cc = c[ll][i];
                cc = fg * cc + ig * gg;
#pragma unroll
                for (int ll = 0; ll < MAXL; ++ll)
                    if (ll == l) c[ll][i] = cc;
                hs[l][cur ^ 1][half * NWH + i][u] = og * tanhf(cc);
            }
            __syncthreads();
        }
        cur ^= 1;
    }
    // last hidden state of the top layer -> BatchNorm (eval affine) -> out
#pragma unroll
    for (int i = 0; i < NWH; ++i) {
        const int w = w0 + half * NWH + i;
        if (w < p.n_win) {
            const float hv = hs[p.L - 1][cur][half * NWH + i][u];
            p.out[(int64_t)w * H + u] = hv * p.out_scale[u] + p.out_shift[u];
        }
    }
}

inline int grid1(int64_t n, int per = 256) {
    int64_t g = (n + per - 1) / per;
    if (g < 1) g = 1;
    return (int)(g < 65536 ? g : 65536);
}

}  // namespace

hipError_t launch_concat_frames(const float* a, int fa, const float* b, int fb, int64_t rows, float* out,
                                hipStream_t s) {
    hipLaunchKernelGGL(concat_frames_kernel, dim3(grid1(rows * (fa + fb))), dim3(256), 0, s, a, fa, b, fb, rows, out);
    return hipGetLastError();
}

hipError_t launch_layernorm_rows(const float* X, int d, int64_t n_rows, int W, int win_stride, const float* pe,
                                 const float* gamma, const float* beta, float eps, float* out, hipStream_t s) {
    if (d > 1024) return hipErrorInvalidValue;
    if (n_rows <= 0) return hipSuccess;
    const auto a16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    if (d % 4 == 0 && d <= 256 && a16(X) && a16(gamma) && a16(beta) && a16(out) && (!pe || a16(pe))) {
        int lpr = 1;
        while (lpr * 4 < d) lpr *= 2;
        constexpr int U = 4;
        const int64_t groups = (n_rows + (64 / lpr) * U - 1) / ((64 / lpr) * U);
        const unsigned wgs = (unsigned)std::min<int64_t>((groups + 3) / 4, 8192);
#define VP3D_LN_VEC(L)                                                                                      \
    case L:                                                                                                 \
        hipLaunchKernelGGL((layernorm_rows_vec_kernel<L, U>), dim3(wgs), dim3(256), 0, s, X, d, n_rows, W, \
                           win_stride, pe, gamma, beta, eps, out);                                          \
        return hipGetLastError();
        switch (lpr) {
            VP3D_LN_VEC(1)
            VP3D_LN_VEC(2)
            VP3D_LN_VEC(4)
            VP3D_LN_VEC(8)
            VP3D_LN_VEC(16)
            VP3D_LN_VEC(32)
            VP3D_LN_VEC(64)
            default: break;
        }
#undef VP3D_LN_VEC
    }
    hipLaunchKernelGGL(layernorm_rows_kernel, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0, s, X, d, n_rows, W,
                       win_stride, pe, gamma, beta, eps, out);
    return hipGetLastError();
}

hipError_t launch_attention(const float* QKV, int n_win, int W, int d, int heads, int last_only, float* O,
                            hipStream_t s) {
    const int dh = d / heads;
    if (dh * heads != d) return hipErrorInvalidValue;
    const float scale = 1.0f / sqrtf((float)dh);
    const size_t smem = (size_t)2 * W * dh * sizeof(float);
    if (smem > 64 * 1024) return hipErrorInvalidValue;
    const dim3 grid(n_win, heads);
    if (last_only && W <= 256 && heads <= 16 && (dh == 16 || dh == 32)) {
        if (dh == 16)
            hipLaunchKernelGGL(attention_last_kernel<16>, dim3(n_win), dim3(64 * heads), 0, s, QKV, W, d, scale, O);
        else
            hipLaunchKernelGGL(attention_last_kernel<32>, dim3(n_win), dim3(64 * heads), 0, s, QKV, W, d, scale, O);
        return hipGetLastError();
    }
    if (!last_only && W <= ATT_WMAX && (dh == 16 || dh == 32)) {
        if (dh == 16)
            hipLaunchKernelGGL(attention_mfma_kernel<16>, grid, dim3(256), 0, s, QKV, W, d, scale, O);
        else
            hipLaunchKernelGGL(attention_mfma_kernel<32>, grid, dim3(256), 0, s, QKV, W, d, scale, O);
        return hipGetLastError();
    }
    switch (dh) {
        case 16: hipLaunchKernelGGL(attention_kernel<16>, grid, dim3(256), smem, s, QKV, W, d, last_only, scale, O); break;
        case 32: hipLaunchKernelGGL(attention_kernel<32>, grid, dim3(256), smem, s, QKV, W, d, last_only, scale, O); break;
        case 64: hipLaunchKernelGGL(attention_kernel<64>, grid, dim3(256), smem, s, QKV, W, d, last_only, scale, O); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_lstm(const LstmParams& p, hipStream_t s) {
    if (p.L < 1 || p.L > LSTM_MAXL) return hipErrorInvalidValue;
    if (p.H == 128 && p.L <= 2) {
        hipLaunchKernelGGL((lstm_kernel<128, 32, 2>), dim3((p.n_win + 31) / 32), dim3(256), 0, s, p);
        return hipGetLastError();
    }
    const dim3 grid((p.n_win + 15) / 16);
    switch (p.H) {
        case 64: hipLaunchKernelGGL((lstm_kernel<64, 16, LSTM_MAXL>), grid, dim3(128), 0, s, p); break;
        case 128: hipLaunchKernelGGL((lstm_kernel<128, 16, LSTM_MAXL>), grid, dim3(256), 0, s, p); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace vp3d
