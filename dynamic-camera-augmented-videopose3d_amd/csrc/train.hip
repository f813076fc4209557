// Training-mode kernels of the temporal conv stack:
// the pieces of one optimisation step of run.py:451-487 (TemporalModel in train
// mode -> mpjpe -> backward -> Adam(amsgrad)) that are not a forward conv GEMM.
//
//   BatchNorm1d, train mode   batch statistics + running-stat update (momentum),
//                             as ATen's CPU kernel forms them (TemporalModel.py:117,119)
//   ReLU + Dropout            TemporalModel.py:130-137 drop(relu(bn(conv(x))))
//   residual add              TemporalModel.py:132,137
//   backward of all of them   (BN backward as ATen's batch_norm_backward)
//   conv weight gradients     dW = dZ^T x gather(X): a TN GEMM over rows, f32 MFMA
//   Adam(amsgrad=True)        torch.optim.Adam single-tensor update, run.py:662
//
// The data are channel-last rows (B*L, C) as everywhere in this library.  All
// arithmetic is f32 (the reference trains in fp32); per-channel reductions are
// accumulated in f64.
#include <climits>
#include "kernels.h"

#pragma clang fp contract(off)

namespace vp3d {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// dropout keep mask: counter-based (splitmix64 of seed, layer, element), so the
// backward regenerates the mask instead of storing it
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool drop_keep(uint64_t seed, int layer, int64_t idx, uint64_t thresh) {
    uint64_t z = seed + (uint64_t)(layer + 1) * 0x9E3779B97F4A7C15ull + (uint64_t)idx * 0xD1B54A32D192ED03ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (z >> 32) < thresh;
}

// ---------------------------------------------------------------------------
// weight packing (per step: the optimiser changes the torch-layout weights)
// ---------------------------------------------------------------------------
__global__ void pack_weights_kernel(const float* __restrict__ w, int cout, int cin, int taps, int mode, int Kp,
                                    float* __restrict__ out) {
    const int64_t total = (int64_t)cout * cin * taps;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int k = (int)(e % taps);
        const int64_t oc = e / taps;
        const int c = (int)(oc % cin);
        const int o = (int)(oc / cin);
        int64_t dst;
        if (mode == 0)  // forward: [o][k*cin + c]
            dst = (int64_t)o * Kp + (int64_t)k * cin + c;
        else if (mode == 1)  // dgrad, flipped taps over a zero-padded gradient: [c][(taps-1-k)*cout + o]
            dst = (int64_t)c * Kp + (int64_t)(taps - 1 - k) * cout + o;
        else  // dgrad, non-overlapping taps (strided / 1x1): [k*cin + c][o]
            dst = ((int64_t)k * cin + c) * Kp + o;
        out[dst] = w[e];
    }
}

// ---------------------------------------------------------------------------
// per-channel column reductions over rows (f64 partial sums per row chunk)
// ---------------------------------------------------------------------------
struct StatsOp {  // BN forward: sum z, sum z^2
    const float* Z;
    int C;
    __device__ void prep(int) {}
    __device__ void operator()(int64_t r, int c, double& a, double& b) const {
        const double z = Z[r * C + c];
        a += z;
        b += z * z;
    }
};

struct SumOp {  // bias gradient: column sum of dy (rows of `ld` elements)
    const float* D;
    int ld;
    __device__ void prep(int) {}
    __device__ void operator()(int64_t r, int c, double& a, double&) const { a += D[r * ld + c]; }
};

// BN backward: g = dOut * keep/(1-p) * [bn(z) > 0];  sums g and g * (z - mean)
struct BnBwdOp {
    const float* dO;
    const float* Z;
    const float* alpha;
    const float* shift;
    const float* mean;
    int C;
    float dscale;
    uint64_t seed, thresh;
    int layer;
    float al, sh, mu;
    __device__ void prep(int c) {
        al = alpha[c];
        sh = shift[c];
        mu = mean[c];
    }
    __device__ void operator()(int64_t r, int c, double& a, double& b) const {
        const int64_t i = r * C + c;
        const float z = Z[i];
        const float y = z * al + sh;
        float g = 0.f;
        if (y > 0.f) {
            g = dO[i];
            if (thresh != (1ull << 32)) g = drop_keep(seed, layer, i, thresh) ? g * dscale : 0.f;
        }
        a += g;
        b += (double)g * (double)(z - mu);
    }
};

template <class Op>
__global__ __launch_bounds__(256) void colreduce_kernel(Op op, int64_t M, int C, int64_t rows_per_chunk,
                                                        double* __restrict__ part) {
    const int c = blockIdx.y * 256 + threadIdx.x;
    if (c >= C) return;
    op.prep(c);
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_chunk;
    const int64_t r1 = min(M, r0 + rows_per_chunk);
    double a0 = 0, b0 = 0, a1 = 0, b1 = 0, a2 = 0, b2 = 0, a3 = 0, b3 = 0;
    int64_t r = r0;
    for (; r + 4 <= r1; r += 4) {
        op(r, c, a0, b0);
        op(r + 1, c, a1, b1);
        op(r + 2, c, a2, b2);
        op(r + 3, c, a3, b3);
    }
    for (; r < r1; ++r) op(r, c, a0, b0);
    part[(int64_t)blockIdx.x * 2 * C + c] = (a0 + a1) + (a2 + a3);
    part[((int64_t)blockIdx.x * 2 + 1) * C + c] = (b0 + b1) + (b2 + b3);
}

__device__ __forceinline__ void sum_parts(const double* part, int nchunks, int C, int c, double& a, double& b) {
    a = 0;
    b = 0;
    for (int k = 0; k < nchunks; ++k) {
        a += part[(int64_t)k * 2 * C + c];
        b += part[((int64_t)k * 2 + 1) * C + c];
    }
}

// batch statistics -> save_mean / save_invstd, the affine (alpha, shift) of the
// transform, running-stat update (ATen batch_norm_cpu_update_stats_template:
// invstd = 1/sqrt(var_biased + eps); running = m * stat + (1 - m) * running,
// running_var with the unbiased variance)
__global__ void bn_finalize_kernel(const double* __restrict__ part, int nchunks, int64_t M, int C,
                                   const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
                                   double momentum, float* running_mean, float* running_var,
                                   float* __restrict__ mean_out, float* __restrict__ invstd_out,
                                   float* __restrict__ alpha_out, float* __restrict__ shift_out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double s, ss;
    sum_parts(part, nchunks, C, c, s, ss);
    const double mean = s / (double)M;
    double var_sum = ss - s * mean;
    if (var_sum < 0) var_sum = 0;
    const float meanf = (float)mean;
    const float invstd = (float)(1.0 / sqrt(var_sum / (double)M + (double)eps));
    const float al = invstd * gamma[c];
    mean_out[c] = meanf;
    invstd_out[c] = invstd;
    alpha_out[c] = al;
    shift_out[c] = beta[c] - meanf * al;
    if (running_mean) {
        running_mean[c] = (float)(momentum * (double)meanf + (1.0 - momentum) * (double)running_mean[c]);
        const double unbiased = M > 1 ? var_sum / (double)(M - 1) : var_sum;
        running_var[c] = (float)(momentum * unbiased + (1.0 - momentum) * (double)running_var[c]);
    }
}

// BN backward coefficients: dgamma = sum(g * xhat), dbeta = sum(g);
// dz = (g - sum(g)/M - (z - mean) * k) * (invstd * gamma),  k = sum(g (z-mean)) invstd^2 / M
__global__ void bn_bwd_finalize_kernel(const double* __restrict__ part, int nchunks, int64_t M, int C,
                                       const float* __restrict__ gamma, const float* __restrict__ invstd,
                                       float* __restrict__ dgamma, float* __restrict__ dbeta,
                                       float* __restrict__ coef /* [3][C]: gmean, k, invstd*gamma */) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double s, dotp;
    sum_parts(part, nchunks, C, c, s, dotp);
    const double is = invstd[c];
    if (dgamma) dgamma[c] = (float)(dotp * is);
    if (dbeta) dbeta[c] = (float)s;
    coef[c] = (float)(s / (double)M);
    coef[C + c] = (float)(dotp * is * is / (double)M);
    coef[2 * C + c] = (float)(is * (double)gamma[c]);
}

__global__ void colsum_finalize_kernel(const double* __restrict__ part, int nchunks, int C, float* __restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double s, unused;
    sum_parts(part, nchunks, C, c, s, unused);
    out[c] = (float)s;
}

// ---------------------------------------------------------------------------
// elementwise passes (float4 over channels; C % 4 == 0)
// ---------------------------------------------------------------------------
// out = [R[res(m)] +] dropout(relu(z * alpha + shift))
__global__ __launch_bounds__(256) void bn_act_fwd_kernel(const float* __restrict__ Z, int64_t M, int C,
                                                         const float* __restrict__ alpha,
                                                         const float* __restrict__ shift, float dscale,
                                                         uint64_t seed, uint64_t thresh, int layer,
                                                         const float* __restrict__ R, int T_out, int R_T,
                                                         int R_stride, int R_off, float* __restrict__ Y) {
    const int c4 = C >> 2;
    const int64_t total = M * c4;
    const bool small = total < INT32_MAX;  // 32-bit row / frame arithmetic
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t m = small ? (int64_t)((uint32_t)e / (uint32_t)c4) : e / c4;
        const int c = (int)(e - m * c4) * 4;
        const f32x4 z = *(const f32x4*)(Z + m * C + c);
        const f32x4 al = *(const f32x4*)(alpha + c);
        const f32x4 sh = *(const f32x4*)(shift + c);
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float v = z[j] * al[j];
            v = v + sh[j];
            v = v > 0.f ? v : 0.f;
            if (thresh != (1ull << 32)) v = drop_keep(seed, layer, m * C + c + j, thresh) ? v * dscale : 0.f;
            o[j] = v;
        }
        if (R) {
            const int64_t b = small ? (int64_t)((uint32_t)m / (uint32_t)T_out) : m / T_out, t = m - b * T_out;
            const f32x4 r = *(const f32x4*)(R + (b * R_T + t * R_stride + R_off) * C + c);
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = r[j] + o[j];
        }
        *(f32x4*)(Y + m * C + c) = o;
    }
}

// dz rows (optionally into a zero-padded row layout: row(m) = b*dz_T + t + dz_off)
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ dO,
                                                           const float* __restrict__ Z, int64_t M, int C,
                                                           const float* __restrict__ alpha,
                                                           const float* __restrict__ shift,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ coef, float dscale,
                                                           uint64_t seed, uint64_t thresh, int layer, int T_out,
                                                           int dz_T, int dz_off, float* __restrict__ dZ) {
    // per-channel operands as float4 (C % 4 == 0, 16-byte aligned: launch_bn_train_backward)
    const int c4 = C >> 2;
    const int64_t total = M * c4;
    const bool small = total < INT32_MAX;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t m = small ? (int64_t)((uint32_t)e / (uint32_t)c4) : e / c4;
        const int c = (int)(e - m * c4) * 4;
        const f32x4 z = *(const f32x4*)(Z + m * C + c);
        const f32x4 d = *(const f32x4*)(dO + m * C + c);
        const f32x4 al = *(const f32x4*)(alpha + c);
        const f32x4 sh = *(const f32x4*)(shift + c);
        const f32x4 mu = *(const f32x4*)(mean + c);
        const f32x4 k0 = *(const f32x4*)(coef + c);
        const f32x4 k1 = *(const f32x4*)(coef + C + c);
        const f32x4 k2 = *(const f32x4*)(coef + 2 * C + c);
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float y = z[j] * al[j] + sh[j];
            float g = 0.f;
            if (y > 0.f) {
                g = d[j];
                if (thresh != (1ull << 32)) g = drop_keep(seed, layer, m * C + c + j, thresh) ? g * dscale : 0.f;
            }
            const float xm = z[j] - mu[j];
            const float v = (g - k0[j]) - xm * k1[j];
            o[j] = v * k2[j];
        }
        const int64_t b = small ? (int64_t)((uint32_t)m / (uint32_t)T_out) : m / T_out, t = m - b * T_out;
        *(f32x4*)(dZ + (b * dz_T + t + dz_off) * C + c) = o;
    }
}

// dIn[b*T_in + t*rs + ro] += dOut[b*T_out + t]  (gradient of the residual slice)
__global__ __launch_bounds__(256) void res_grad_add_kernel(float* __restrict__ dIn, const float* __restrict__ dOut,
                                                           int64_t M, int C, int T_out, int T_in, int rs, int ro) {
    const int c4 = C >> 2;
    const int64_t total = M * c4;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t m = e / c4;
        const int c = (int)(e - m * c4) * 4;
        const int64_t b = m / T_out, t = m - b * T_out;
        f32x4* dst = (f32x4*)(dIn + (b * T_in + t * rs + ro) * C + c);
        const f32x4 g = *(const f32x4*)(dOut + m * C + c);
        f32x4 v = *dst;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = v[j] + g[j];
        *dst = v;
    }
}

// ---------------------------------------------------------------------------
// weight gradient: part[s][n][k] = sum_{m in split s} dZ[dzrow(m)][n] * X[src(m) + tap*dil][c],
// k = tap*cin + c.  128x128 output tile per workgroup (4 waves of 64x64), rows
// streamed 16 at a time through LDS (double buffered, register prefetch), f32 MFMA
// 16x16x4: the contraction index (rows) runs down the lanes' k slot, so both
// operands are read from m-major LDS rows without a transpose.
// ---------------------------------------------------------------------------
constexpr int WG_T = 128;      // tile edge (n and k)
constexpr int WG_R = 16;       // rows per stage
constexpr int WG_LD = 128 + 16; // LDS row pitch (floats): 4 rows start 16 banks apart

__device__ __forceinline__ float4 ld4_or_zero(const float* p, bool ok) {
    return ok ? *(const float4*)p : make_float4(0.f, 0.f, 0.f, 0.f);
}

__global__ __launch_bounds__(256) void wgrad_f32_kernel(WgradParams p) {
    __shared__ __attribute__((aligned(16))) float sm[2][2][WG_R * WG_LD];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int ntn = (p.N + WG_T - 1) / WG_T;
    const int tile_n = blockIdx.x % ntn, tile_k = blockIdx.x / ntn;
    const int n0 = tile_n * WG_T, k0 = tile_k * WG_T;
    const int64_t mb = (int64_t)blockIdx.y * p.rows_per_split;
    const int64_t me = min((int64_t)p.M, mb + p.rows_per_split);

    // loader: thread -> (row lr = tid/32 + 8*i, 4 columns at c4 = (tid%32)*4), i = 0, 1
    const int lr = tid >> 5, lc = (tid & 31) * 4;
    const bool nvec = (p.N % 4 == 0) && (n0 + lc + 3 < p.N);
    const int kk = k0 + lc;
    const int tapv = kk / p.cin, cv = kk - tapv * p.cin;
    const bool kvec = (p.cin % 4 == 0) && (kk + 3 < p.K);
    float4 ra[2], rb[2];

    auto gload = [&](int64_t m0) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int64_t m = m0 + lr + 8 * i;
            const bool mv = m < me;
            int64_t b = 0, t = 0;
            if (mv) {
                b = m / p.T_out;
                t = m - b * p.T_out;
            }
            const float* dzr = p.dZ + (b * p.dz_T + t + p.dz_off) * (int64_t)p.ldz;
            if (nvec) {
                ra[i] = ld4_or_zero(dzr + n0 + lc, mv);
            } else {
                float v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = (mv && n0 + lc + j < p.N) ? dzr[n0 + lc + j] : 0.f;
                ra[i] = make_float4(v[0], v[1], v[2], v[3]);
            }
            const int64_t srow = b * p.T_in + t * p.stride;
            if (kvec) {
                rb[i] = ld4_or_zero(p.X + (srow + (int64_t)tapv * p.dil) * p.cin + cv, mv);
            } else {
                float v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int k = kk + j;
                    float x = 0.f;
                    if (mv && k < p.K) {
                        const int tap = k / p.cin, c = k - tap * p.cin;
                        x = p.X[(srow + (int64_t)tap * p.dil) * p.cin + c];
                    }
                    v[j] = x;
                }
                rb[i] = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            *(float4*)&sm[buf][0][(lr + 8 * i) * WG_LD + lc] = ra[i];
            *(float4*)&sm[buf][1][(lr + 8 * i) * WG_LD + lc] = rb[i];
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int wn = (wid >> 1) * 64, wk = (wid & 1) * 64;
    const int fr = lane >> 4, fc = lane & 15;
    if (mb < me) {
        gload(mb);
        lstore(0);
    }
    __syncthreads();
    int cur = 0;
    for (int64_t m0 = mb; m0 < me; m0 += WG_R) {
        const bool more = m0 + WG_R < me;
        if (more) gload(m0 + WG_R);
        const float* As = sm[cur][0];
        const float* Bs = sm[cur][1];
#pragma unroll
        for (int s = 0; s < WG_R / 4; ++s) {
            float af[4], bfr[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i] = As[(s * 4 + fr) * WG_LD + wn + i * 16 + fc];
#pragma unroll
            for (int j = 0; j < 4; ++j) bfr[j] = Bs[(s * 4 + fr) * WG_LD + wk + j * 16 + fc];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
        if (more) lstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }

    float* out = p.part + (int64_t)blockIdx.y * p.N * (int64_t)p.K;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = n0 + wn + i * 16 + fr * 4 + r;
                const int k = k0 + wk + j * 16 + fc;
                if (n < p.N && k < p.K) out[(int64_t)n * p.K + k] = acc[i][j][r];
            }
}

// dW (torch layout (N, cin, taps)) = sum over splits of part[s][n][tap*cin + c]
__global__ void wgrad_reduce_kernel(const float* __restrict__ part, int S, int N, int K, int cin, int taps,
                                    float* __restrict__ dW) {
    const int64_t total = (int64_t)N * K;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        float s = 0.f;
        for (int i = 0; i < S; ++i) s += part[(int64_t)i * total + e];
        const int n = (int)(e / K);
        const int k = (int)(e - (int64_t)n * K);
        const int tap = k / cin, c = k - tap * cin;
        dW[((int64_t)n * cin + c) * taps + tap] = s;
    }
}

// ---------------------------------------------------------------------------
// Adam (torch.optim.Adam, _single_tensor_adam), one launch for a list of tensors
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void adam_kernel(AdamList L, AdamHyper hp) {
    int t = 0;
    while (t + 1 < L.n && (int)blockIdx.x >= L.block_start[t + 1]) ++t;
    const int64_t n = L.numel[t];
    float* __restrict__ p = L.param[t];
    const float* __restrict__ g = L.grad[t];
    float* __restrict__ m = L.exp_avg[t];
    float* __restrict__ v = L.exp_avg_sq[t];
    float* __restrict__ vmax = L.max_exp_avg_sq[t];
    const int64_t base = (int64_t)(blockIdx.x - L.block_start[t]) * 256 * 4;
    for (int j = 0; j < 4; ++j) {
        const int64_t i = base + j * 256 + threadIdx.x;
        if (i >= n) break;
        float gi = g[i];
        const float pi = p[i];
        if (hp.weight_decay != 0.f) gi = gi + pi * hp.weight_decay;  // grad.add(param, alpha=wd)
        // exp_avg.lerp_(grad, 1 - beta1): ATen lerp, |w| < 0.5 branch
        float mi = m[i];
        // (ATen's vectorised lerp: fmadd(coeff, end - start, base))
        mi = hp.lerp_w < 0.5f ? __builtin_fmaf(hp.lerp_w, gi - mi, mi) : __builtin_fmaf(hp.lerp_w - 1.f, gi - mi, gi);
        // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
        // (ATen's vectorised addcmul: fmadd(value * t1, t2, self))
        float vi = v[i] * hp.beta2;
        vi = __builtin_fmaf(hp.one_minus_beta2 * gi, gi, vi);
        float denom;
        if (hp.amsgrad) {
            float vm = vmax[i];
            vm = vm > vi ? vm : vi;  // torch.maximum
            vmax[i] = vm;
            denom = __builtin_sqrtf(vm) / hp.bc2_sqrt + hp.eps;
        } else {
            denom = __builtin_sqrtf(vi) / hp.bc2_sqrt + hp.eps;
        }
        m[i] = mi;
        v[i] = vi;
        p[i] = pi + hp.neg_step_size * mi / denom;  // addcdiv_(exp_avg, denom, value=-step_size)
    }
}

__global__ void relu_mask_kernel(const float* __restrict__ Z, int64_t n, int C, const float* __restrict__ alpha,
                                 const float* __restrict__ shift, uint8_t* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        out[i] = (Z[i] * alpha[c] + shift[c]) > 0.f ? 1 : 0;
    }
}

__global__ void dropout_mask_kernel(uint64_t seed, uint64_t thresh, int layer, int64_t n, uint8_t* out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = thresh == (1ull << 32) ? 1 : (drop_keep(seed, layer, i, thresh) ? 1 : 0);
}

inline int grid_for(int64_t work, int per_block = 256, int cap = 65536) {
    int64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    return (int)(g < cap ? g : cap);
}

inline uint64_t keep_threshold(float p) {
    if (p <= 0.f) return 1ull << 32;
    const double keep = 1.0 - (double)p;
    return (uint64_t)(keep * 4294967296.0);
}

// rows per chunk of a column reduction: enough chunks to fill the chip, >= 64 rows each
int64_t reduce_rows(int64_t M, int C) {
    const int cgroups = (C + 255) / 256;
    int64_t chunks = (2048 + cgroups - 1) / cgroups;
    int64_t rows = (M + chunks - 1) / chunks;
    if (rows < 64) rows = 64;
    return rows;
}

template <class Op>
hipError_t launch_colreduce(const Op& op, int64_t M, int C, double* part, int* nchunks, hipStream_t s) {
    const int64_t rows = reduce_rows(M, C);
    const int64_t nc = M > 0 ? (M + rows - 1) / rows : 1;
    *nchunks = (int)nc;
    if (M == 0) {
        (void)hipMemsetAsync(part, 0, sizeof(double) * 2 * C, s);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(colreduce_kernel<Op>, dim3((unsigned)nc, (C + 255) / 256), dim3(256), 0, s, op, M, C, rows,
                       part);
    return hipGetLastError();
}

}  // namespace

int64_t train_reduce_part_doubles(int64_t M, int C) {
    const int64_t rows = reduce_rows(M, C);
    const int64_t nc = M > 0 ? (M + rows - 1) / rows : 1;
    return nc * 2 * C;
}

hipError_t launch_pack_weights(const float* w, int cout, int cin, int taps, int mode, int Kp, float* out,
                               hipStream_t s) {
    const int64_t total = (int64_t)cout * cin * taps;
    hipLaunchKernelGGL(pack_weights_kernel, dim3(grid_for(total)), dim3(256), 0, s, w, cout, cin, taps, mode, Kp,
                       out);
    return hipGetLastError();
}

hipError_t launch_bn_train_stats(const float* Z, int64_t M, int C, double* part, const float* gamma,
                                 const float* beta, float eps, double momentum, float* running_mean,
                                 float* running_var, float* mean, float* invstd, float* alpha, float* shift,
                                 hipStream_t s) {
    int nc = 0;
    hipError_t e = launch_colreduce(StatsOp{Z, C}, M, C, part, &nc, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, s, part, nc, M, C, gamma, beta, eps,
                       momentum, running_mean, running_var, mean, invstd, alpha, shift);
    return hipGetLastError();
}

hipError_t launch_bn_act_fwd(const float* Z, int64_t M, int C, const float* alpha, const float* shift, float p,
                             uint64_t seed, int layer, const float* R, int T_out, int R_T, int R_stride, int R_off,
                             float* Y, hipStream_t s) {
    const float dscale = p > 0.f ? 1.0f / (float)(1.0 - (double)p) : 1.0f;
    hipLaunchKernelGGL(bn_act_fwd_kernel, dim3(grid_for(M * (C / 4))), dim3(256), 0, s, Z, M, C, alpha, shift, dscale,
                       seed, keep_threshold(p), layer, R, T_out, R_T, R_stride, R_off, Y);
    return hipGetLastError();
}

hipError_t launch_bn_train_backward(const float* dO, const float* Z, int64_t M, int C, const float* gamma,
                                    const float* alpha, const float* shift, const float* mean, const float* invstd,
                                    float p, uint64_t seed, int layer, double* part, float* coef, float* dgamma,
                                    float* dbeta, int T_out, int dz_T, int dz_off, float* dZ, hipStream_t s) {
    const float dscale = p > 0.f ? 1.0f / (float)(1.0 - (double)p) : 1.0f;
    const uint64_t thresh = keep_threshold(p);
    BnBwdOp op{dO, Z, alpha, shift, mean, C, dscale, seed, thresh, layer};
    int nc = 0;
    hipError_t e = launch_colreduce(op, M, C, part, &nc, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, s, part, nc, M, C, gamma, invstd,
                       dgamma, dbeta, coef);
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for(M * (C / 4))), dim3(256), 0, s, dO, Z, M, C, alpha, shift,
                       mean, coef, dscale, seed, thresh, layer, T_out, dz_T, dz_off, dZ);
    return hipGetLastError();
}

hipError_t launch_colsum(const float* D, int64_t M, int C, int ld, double* part, float* out, hipStream_t s) {
    int nc = 0;
    hipError_t e = launch_colreduce(SumOp{D, ld}, M, C, part, &nc, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(colsum_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, s, part, nc, C, out);
    return hipGetLastError();
}

hipError_t launch_res_grad_add(float* dIn, const float* dOut, int64_t M, int C, int T_out, int T_in, int rs, int ro,
                               hipStream_t s) {
    hipLaunchKernelGGL(res_grad_add_kernel, dim3(grid_for(M * (C / 4))), dim3(256), 0, s, dIn, dOut, M, C, T_out, T_in,
                       rs, ro);
    return hipGetLastError();
}

int wgrad_splits(int64_t M, int N, int K, int64_t max_part_floats) {
    const int64_t tiles = (int64_t)((N + WG_T - 1) / WG_T) * ((K + WG_T - 1) / WG_T);
    int64_t S = (2048 + tiles - 1) / tiles;
    const int64_t by_rows = (M + 255) / 256;  // at least 256 rows per split
    if (S > by_rows) S = by_rows;
    const int64_t by_mem = max_part_floats / ((int64_t)N * K);
    if (S > by_mem) S = by_mem;
    if (S < 1) S = 1;
    return (int)S;
}

hipError_t launch_wgrad(const WgradParams& p0, int S, int taps, float* dW, hipStream_t s) {
    WgradParams p = p0;
    const int64_t rps = (p.M + S - 1) / S;
    p.rows_per_split = (rps + WG_R - 1) / WG_R * WG_R;
    const int tiles = ((p.N + WG_T - 1) / WG_T) * ((p.K + WG_T - 1) / WG_T);
    hipLaunchKernelGGL(wgrad_f32_kernel, dim3(tiles, S), dim3(256), 0, s, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(grid_for((int64_t)p.N * p.K)), dim3(256), 0, s, p.part, S, p.N, p.K,
                       p.cin, taps, dW);
    return hipGetLastError();
}

hipError_t launch_adam(const AdamList& L, const AdamHyper& hp, hipStream_t s) {
    if (L.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(adam_kernel, dim3(L.block_start[L.n]), dim3(256), 0, s, L, hp);
    return hipGetLastError();
}

hipError_t launch_relu_mask(const float* Z, int64_t n, int C, const float* alpha, const float* shift, uint8_t* out,
                            hipStream_t s) {
    hipLaunchKernelGGL(relu_mask_kernel, dim3(grid_for(n)), dim3(256), 0, s, Z, n, C, alpha, shift, out);
    return hipGetLastError();
}

hipError_t launch_dropout_mask(uint64_t seed, float p, int layer, int64_t n, uint8_t* out, hipStream_t s) {
    hipLaunchKernelGGL(dropout_mask_kernel, dim3(grid_for(n)), dim3(256), 0, s, seed, keep_threshold(p), layer, n, out);
    return hipGetLastError();
}

}  // namespace vp3d
