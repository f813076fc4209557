// On-device input path of the lifter (HBM-bound element/gather kernels).
//
//   normalize_screen   reference common/camera.py:14-18 (+ inverse, :21-25)
//   camera_matrices    reference common/generators.py:115-125, :180-190 (K @ E_t)
//   world_to_camera    reference common/camera.py:28-30, common/quaternion.py:10-35
//   gather_windows     reference common/generators.py:92-137 (pad_chunk, 'edge'),
//                      :193-198, fused with the trajectory concat of
//                      common/models/CamTransformer.py:187-190
//   mpjpe_accumulate   reference common/loss.py:11-17
//   project_to_2d      reference common/camera.py:37-67 (H36M distortion), :69-90 (linear)
//
// Floating-point contraction is OFF (build flag -ffp-contract=off, plus the pragma
// below): HIP compiles with -ffp-contract=fast by default and __fadd_rn/__fmul_rn
// are plain operators, so a mul followed by an add would silently become an FMA.  The reference evaluates
// these formulas as separately rounded numpy / torch-CPU operations; the kernels
// spell out exactly that rounding sequence (and use __builtin_fmaf only where
// torch's own CPU kernel fuses), which makes them bit-exact on the goldens.
#include "kernels.h"

#pragma clang fp contract(off)

namespace vp3d {
namespace {

constexpr int kThreads = 256;

inline dim3 grid_for(int64_t n, int per_thread = 1) {
    int64_t blocks = (n + (int64_t)kThreads * per_thread - 1) / ((int64_t)kThreads * per_thread);
    if (blocks < 1) blocks = 1;
    if (blocks > 65535 * 16) blocks = 65535 * 16;
    return dim3((unsigned)blocks);
}

// X/w*2 - [1, h/w]: numpy evaluates X/w and *2 in float32 (array op with a
// Python int), then subtracts a float64 list, i.e. in float64, and run.py
// stores the float64 result back into a float32 array (one final rounding).
__global__ void normalize_screen_kernel(const float* __restrict__ x, int64_t n, float wf,
                                        double hw, float* __restrict__ out, int inverse,
                                        float halfw) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float2 v = reinterpret_cast<const float2*>(x)[i];
        float2 r;
        if (!inverse) {
            const float a = __fmul_rn(__fdiv_rn(v.x, wf), 2.0f);
            const float b = __fmul_rn(__fdiv_rn(v.y, wf), 2.0f);
            r.x = (float)__dsub_rn((double)a, 1.0);
            r.y = (float)__dsub_rn((double)b, hw);
        } else {
            // (X + [1, h/w]) * w / 2: float64 add (list promotion), then *w and /2 in float64
            r.x = (float)__ddiv_rn(__dmul_rn(__dadd_rn((double)v.x, 1.0), (double)wf), 2.0);
            r.y = (float)__ddiv_rn(__dmul_rn(__dadd_rn((double)v.y, hw), (double)wf), 2.0);
        }
        reinterpret_cast<float2*>(out)[i] = r;
        (void)halfw;
    }
}

// float64 keypoints (3DPW): X / w * 2 - [1, hw] entirely in float64, rounded once
__global__ void normalize_screen_f64_kernel(const double* __restrict__ x, int64_t n, double w, double hw,
                                            float* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double2 v = reinterpret_cast<const double2*>(x)[i];
        float2 r;
        r.x = (float)__dsub_rn(__dmul_rn(__ddiv_rn(v.x, w), 2.0), 1.0);
        r.y = (float)__dsub_rn(__dmul_rn(__ddiv_rn(v.y, w), 2.0), hw);
        reinterpret_cast<float2*>(out)[i] = r;
    }
}

// K (float32, from the sequence's intrinsics) @ E_t (float64) in float64,
// rounded once to float32 when run.py casts the batch (`astype('float32')`).
// K = [[fx,0,cx],[0,fy,cy],[0,0,1]] so each entry has at most two non-zero
// products; their sum is order-independent, hence bit-exact.
__global__ void camera_matrices_kernel(const float* __restrict__ intr,
                                       const int32_t* __restrict__ frame_seq,
                                       const double* __restrict__ extr, int64_t n,
                                       float* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * 12;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t f = i / 12;
        const int e = (int)(i - f * 12);
        const int row = e >> 2, col = e & 3;
        const float* K = intr + 4 * (int64_t)frame_seq[f];
        const double* E = extr + 12 * f;
        double v;
        if (row == 0)
            v = __dadd_rn(__dmul_rn((double)K[0], E[col]), __dmul_rn((double)K[2], E[8 + col]));
        else if (row == 1)
            v = __dadd_rn(__dmul_rn((double)K[1], E[4 + col]), __dmul_rn((double)K[3], E[8 + col]));
        else
            v = E[8 + col];
        out[i] = (float)v;
    }
}

// qrot(q, v) = v + 2 * (w * (q_xyz x v) + q_xyz x (q_xyz x v)), q = qinverse(R).
__global__ void world_to_camera_kernel(const float* __restrict__ X, int64_t n, float qw,
                                       float qx, float qy, float qz, float tx, float ty,
                                       float tz, float* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float vx = __fsub_rn(X[3 * i + 0], tx);
        const float vy = __fsub_rn(X[3 * i + 1], ty);
        const float vz = __fsub_rn(X[3 * i + 2], tz);
        // uv = cross(qvec, v), uuv = cross(qvec, uv): torch-CPU's cross kernel
        // evaluates each component as fma(a1, b2, -(a2 * b1)) (reproduced bit for
        // bit on the golden vectors), the rest are separately rounded tensor ops.
        const float uvx = __builtin_fmaf(qy, vz, -__fmul_rn(qz, vy));
        const float uvy = __builtin_fmaf(qz, vx, -__fmul_rn(qx, vz));
        const float uvz = __builtin_fmaf(qx, vy, -__fmul_rn(qy, vx));
        const float uuvx = __builtin_fmaf(qy, uvz, -__fmul_rn(qz, uvy));
        const float uuvy = __builtin_fmaf(qz, uvx, -__fmul_rn(qx, uvz));
        const float uuvz = __builtin_fmaf(qx, uvy, -__fmul_rn(qy, uvx));
        out[3 * i + 0] = __fadd_rn(vx, __fmul_rn(2.f, __fadd_rn(__fmul_rn(qw, uvx), uuvx)));
        out[3 * i + 1] = __fadd_rn(vy, __fmul_rn(2.f, __fadd_rn(__fmul_rn(qw, uvy), uuvy)));
        out[3 * i + 2] = __fadd_rn(vz, __fmul_rn(2.f, __fadd_rn(__fmul_rn(qw, uvz), uuvz)));
    }
}

// One thread per output element (b, t, c) of the (B, window, F2 [+12]) window
// tensor; consecutive threads walk c, so reads of one frame's keypoints and
// writes of one window row are contiguous.
__global__ void gather_windows_kernel(const float* __restrict__ kps, int f2,
                                      const float* __restrict__ cams,
                                      const int64_t* __restrict__ seq_off,
                                      const int32_t* __restrict__ seq_len,
                                      const int32_t* __restrict__ pairs, int B, int window,
                                      int lead, float* __restrict__ out) {
    const int fo = f2 + (cams ? 12 : 0);
    const int64_t total = (int64_t)B * window * fo;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t bt = i / fo;
        const int c = (int)(i - bt * fo);
        const int b = (int)(bt / window);
        const int t = (int)(bt - (int64_t)b * window);
        const int seq = pairs[2 * b];
        const int len = seq_len[seq];
        int f = pairs[2 * b + 1] - lead + t;
        f = f < 0 ? 0 : (f >= len ? len - 1 : f);
        const int64_t frame = seq_off[seq] + f;
        out[i] = (c < f2) ? kps[frame * f2 + c] : cams[frame * 12 + (c - f2)];
    }
}

// Block-reduced sum of per-joint Euclidean distances in float64.
__global__ void mpjpe_kernel(const float* __restrict__ pred, const float* __restrict__ target,
                             int64_t n, double* __restrict__ acc) {
    double s = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float dx = pred[3 * i] - target[3 * i];
        const float dy = pred[3 * i + 1] - target[3 * i + 1];
        const float dz = pred[3 * i + 2] - target[3 * i + 2];
        s += sqrt((double)dx * dx + (double)dy * dy + (double)dz * dz);
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    __shared__ double part[kThreads / 64];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < kThreads / 64; ++w) t += part[w];
        atomicAdd(acc, t);
        if (blockIdx.x == 0) atomicAdd(acc + 1, (double)n);
    }
}

// Gradient of mpjpe = mean ||pred - target|| (loss.py:11-17) wrt pred, the backward of
// torch.mean(torch.norm(d, dim=-1)): g/n * d / ||d|| per point (0 where ||d|| == 0, as
// torch's norm backward masks it).  g = *grad_loss (device scalar).
__global__ void mpjpe_backward_kernel(const float* __restrict__ pred, const float* __restrict__ target,
                                      int64_t n, const float* __restrict__ grad_loss,
                                      float* __restrict__ grad_pred) {
    const float gn = grad_loss[0] / (float)n;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float dx = pred[3 * i] - target[3 * i];
        const float dy = pred[3 * i + 1] - target[3 * i + 1];
        const float dz = pred[3 * i + 2] - target[3 * i + 2];
        const float nrm = sqrtf(dx * dx + dy * dy + dz * dz);
        const float sc = nrm > 0.f ? gn / nrm : 0.f;
        grad_pred[3 * i] = dx * sc;
        grad_pred[3 * i + 1] = dy * sc;
        grad_pred[3 * i + 2] = dz * sc;
    }
}

// H36M camera projection of camera-space points, one thread per point; camera of
// point i = i / pts_per_cam, params [f(2), c(2), k(3), p(2)].  The torch-float32
// op order of camera.py:59-67: XX = clamp(X_xy / X_z, -1, 1); r2 = (0 + x^2) + y^2;
// radial = 1 + (((0 + k1 r2) + k2 r2^2) + k3 r2^3) with r2^3 = (r2 r2) r2 (ATen's pow
// for exponent 3); tan = (0 + p1 x) + p2 y; out = f * (XX (radial + tan) + p r2) + c.
__global__ void project_to_2d_kernel(const float* __restrict__ X, int64_t n, int64_t pts_per_cam,
                                     const float* __restrict__ prm, int linear, float* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float* q = prm + (i / pts_per_cam) * 9;
        const float z = X[3 * i + 2];
        float u = X[3 * i] / z, v = X[3 * i + 1] / z;
        u = fminf(fmaxf(u, -1.f), 1.f);
        v = fminf(fmaxf(v, -1.f), 1.f);
        float ox = u, oy = v;
        if (!linear) {
            const float r2 = u * u + v * v;
            const float r4 = r2 * r2;
            const float r6 = r4 * r2;
            const float radial = 1.f + ((q[4] * r2 + q[5] * r4) + q[6] * r6);
            const float tan = q[7] * u + q[8] * v;
            ox = u * (radial + tan) + q[7] * r2;
            oy = v * (radial + tan) + q[8] * r2;
        }
        out[2 * i] = q[0] * ox + q[2];
        out[2 * i + 1] = q[1] * oy + q[3];
    }
}

}  // namespace

hipError_t launch_project_to_2d(const float* X, int64_t n_cams, int64_t pts_per_cam, const float* params,
                                bool linear, float* out, hipStream_t s) {
    const int64_t n = n_cams * pts_per_cam;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(project_to_2d_kernel, grid_for(n, 4), dim3(kThreads), 0, s, X, n, pts_per_cam, params,
                       linear ? 1 : 0, out);
    return hipGetLastError();
}

hipError_t launch_normalize_screen(const float* x, int64_t n, int w, int h, float* out,
                                   bool inverse, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const double hw = (double)h / (double)w;
    hipLaunchKernelGGL(normalize_screen_kernel, grid_for(n, 4), dim3(kThreads), 0, s, x, n,
                       (float)w, hw, out, inverse ? 1 : 0, 0.f);
    return hipGetLastError();
}

hipError_t launch_normalize_screen_f64(const double* x, int64_t n, double w, double hw, float* out,
                                       hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(normalize_screen_f64_kernel, grid_for(n, 4), dim3(kThreads), 0, s, x, n, w, hw, out);
    return hipGetLastError();
}

hipError_t launch_camera_matrices(const float* intr, const int32_t* frame_seq, const double* extr,
                                  int64_t n_frames, float* out, hipStream_t s) {
    if (n_frames <= 0) return hipSuccess;
    hipLaunchKernelGGL(camera_matrices_kernel, grid_for(n_frames * 12, 4), dim3(kThreads), 0, s,
                       intr, frame_seq, extr, n_frames, out);
    return hipGetLastError();
}

hipError_t launch_world_to_camera(const float* X, int64_t n, const float q[4], const float t[3],
                                  float* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    // qinverse (quaternion.py:27-35): (w, -x, -y, -z)
    hipLaunchKernelGGL(world_to_camera_kernel, grid_for(n, 4), dim3(kThreads), 0, s, X, n, q[0],
                       -q[1], -q[2], -q[3], t[0], t[1], t[2], out);
    return hipGetLastError();
}

hipError_t launch_gather_windows(const float* kps, int f2, const float* cams,
                                 const int64_t* seq_off, const int32_t* seq_len,
                                 const int32_t* pairs, int B, int window, int pad, int shift,
                                 float* out, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    const int64_t total = (int64_t)B * window * (f2 + (cams ? 12 : 0));
    hipLaunchKernelGGL(gather_windows_kernel, grid_for(total, 4), dim3(kThreads), 0, s, kps, f2,
                       cams, seq_off, seq_len, pairs, B, window, pad + shift, out);
    return hipGetLastError();
}

hipError_t launch_mpjpe_backward(const float* pred, const float* target, int64_t n, const float* grad_loss,
                                 float* grad_pred, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(mpjpe_backward_kernel, grid_for(n, 1), dim3(kThreads), 0, s, pred, target, n, grad_loss,
                       grad_pred);
    return hipGetLastError();
}

hipError_t launch_mpjpe_accumulate(const float* pred, const float* target, int64_t n,
                                   double* acc, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(mpjpe_kernel, grid_for(n, 8), dim3(kThreads), 0, s, pred, target, n, acc);
    return hipGetLastError();
}

}  // namespace vp3d

namespace vp3d {
namespace {

// Row packer for the first (expand) convolution on the 16-bit path: the
// channel-last f32 input rows that one output frame reads (w0 consecutive frames
// of J*F values, TemporalModel.py:102/168) become one zero-padded 16-bit GEMM row
// of Kp elements, so that layer runs on the tap-aligned LDS-DMA kernel.
template <typename CT>
__global__ void pack_rows_kernel(const float* __restrict__ x, int M, int T_out, int T_in,
                                 int stride, int lda, int K, int Kp, CT* __restrict__ out) {
    const int chunks = Kp >> 3;
    const int64_t total = (int64_t)M * chunks;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int m = (int)(i / chunks);
        const int c = (int)(i - (int64_t)m * chunks) * 8;
        const int b = m / T_out;
        const int t = m - b * T_out;
        const float* row = x + ((int64_t)b * T_in + (int64_t)t * stride) * lda;
        typedef CT ct8 __attribute__((ext_vector_type(8)));
        ct8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (CT)(c + e < K ? row[c + e] : 0.f);
        *(ct8*)(out + (int64_t)m * Kp + c) = v;
    }
}

// Split-fp16 expand rows (VP3D_DTYPE_F16X3): 8 K values per thread -> 16 B of hi and,
// 64 B further, 16 B of lo.  With `pairs` the frames come straight from the sequences,
// edge-clamped per sequence as gather_windows_kernel (generators.py:92-137), each
// frame = [kps (f2) | cams (12)] (CamTransformer.py:187-190).
__global__ void pack_rows_x3_kernel(const float* __restrict__ x, const float* __restrict__ kps, int f2,
                                    const float* __restrict__ cams, const int64_t* __restrict__ seq_off,
                                    const int32_t* __restrict__ seq_len, const int32_t* __restrict__ pairs,
                                    int lead, int M, int T_out, int T_in, int stride, int cin, int K, int Kp,
                                    _Float16* __restrict__ out, unsigned* fault) {
    const int chunks = Kp >> 3;
    bool ok = true;  // every hi half finite (a value past the f16 range or a NaN: not), else kFaultNonFinite
    const int64_t total = (int64_t)M * chunks;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int m = (int)(i / chunks);
        const int c = (int)(i - (int64_t)m * chunks) * 8;
        const int b = m / T_out;
        const int t = m - b * T_out;
        float v[8];
        if (pairs) {
            const int seq = pairs[2 * b];
            const int len = seq_len[seq];
            const int f0 = pairs[2 * b + 1] - lead + t * stride;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int k = c + e;
                v[e] = 0.f;
                if (k < K) {
                    const int tap = k / cin;
                    const int ch = k - tap * cin;
                    int f = f0 + tap;
                    f = f < 0 ? 0 : (f >= len ? len - 1 : f);
                    const int64_t frame = seq_off[seq] + f;
                    v[e] = ch < f2 ? kps[frame * f2 + ch] : cams[frame * 12 + (ch - f2)];
                }
            }
        } else {
            const float* row = x + ((int64_t)b * T_in + (int64_t)t * stride) * cin;
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = c + e < K ? row[c + e] : 0.f;
        }
        typedef _Float16 h8 __attribute__((ext_vector_type(8)));
        h8 hi, lo;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            hi[e] = (_Float16)v[e];
            lo[e] = (_Float16)(v[e] - (float)hi[e]);
            ok = ok && !((__builtin_bit_cast(unsigned short, hi[e]) & 0x7FFFu) >= 0x7C00u);  // inf / NaN hi
        }
        _Float16* o = out + (int64_t)m * 2 * Kp + (c >> 5) * 64 + (c & 31);
        *(h8*)o = hi;
        *(h8*)(o + 32) = lo;
    }
    if (!ok && fault) __hip_atomic_fetch_or(fault, kFaultNonFinite, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

hipError_t launch_pack_rows_x3(const float* x, const GatherSrc* g, int M, int T_out, int T_in, int stride,
                               int cin, int K, int Kp, void* out, unsigned* fault, hipStream_t s) {
    if (M <= 0) return hipSuccess;
    const dim3 grid = grid_for((int64_t)M * (Kp / 8), 4);
    if (g)
        hipLaunchKernelGGL(pack_rows_x3_kernel, grid, dim3(kThreads), 0, s, nullptr, g->kps, g->f2, g->cams,
                           g->seq_off, g->seq_len, g->pairs, g->lead, M, T_out, T_in, stride, cin, K, Kp,
                           (_Float16*)out, fault);
    else
        hipLaunchKernelGGL(pack_rows_x3_kernel, grid, dim3(kThreads), 0, s, x, nullptr, 0, nullptr, nullptr,
                           nullptr, nullptr, 0, M, T_out, T_in, stride, cin, K, Kp, (_Float16*)out, fault);
    return hipGetLastError();
}

hipError_t launch_pack_rows(const float* x, int M, int T_out, int T_in, int stride, int lda,
                            int K, int Kp, void* out, bool bf16, hipStream_t s) {
    if (M <= 0) return hipSuccess;
    const dim3 grid = grid_for((int64_t)M * (Kp / 8), 4);
    if (bf16)
        hipLaunchKernelGGL(pack_rows_kernel<__bf16>, grid, dim3(kThreads), 0, s, x, M, T_out, T_in,
                           stride, lda, K, Kp, (__bf16*)out);
    else
        hipLaunchKernelGGL(pack_rows_kernel<_Float16>, grid, dim3(kThreads), 0, s, x, M, T_out, T_in,
                           stride, lda, K, Kp, (_Float16*)out);
    return hipGetLastError();
}

}  // namespace vp3d
