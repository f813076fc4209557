// Evaluation metrics of the lifter's output, on device:
//
//   MPJPE               reference common/loss.py:11-17   (Protocol #1)
//   P-MPJPE             reference common/loss.py:29-68   (Protocol #2: rigid alignment with
//                       scale, rotation and translation per frame)
//   N-MPJPE             reference common/loss.py:70-80   (per-frame scale only)
//   MPJVE               reference common/loss.py:82-91   (first difference along frames)
//
// One thread per frame of a (n_frames, J, 3) pair of pose arrays, float64 throughout,
// block-reduced partial sums added to a device accumulator (six doubles):
//   acc[0] += sum of per-joint errors          acc[4] += n_frames * J
//   acc[1] += sum of aligned per-joint errors  acc[5] += (n_frames - 1) * J
//   acc[2] += sum of scaled per-joint errors
//   acc[3] += sum of per-joint velocity errors
// so MPJPE = acc0/acc4, P-MPJPE = acc1/acc4, N-MPJPE = acc2/acc4, MPJVE = acc3/acc5
// (every frame has J joints, so the reference's mean of per-frame means is the same).
//
// Rotation of P-MPJPE.  The reference takes np.linalg.svd(H), H = X0^T Y0 of the
// centred, norm-scaled poses, forms R = V U^T and, when det R < 0, negates the last
// singular vector and singular value; the scale is (s1 + s2 + sign(det) s3) normX/normY.
// That reflection-corrected R is the best PROPER rotation taking the prediction onto
// the target, and s1 + s2 + sign(det) s3 is the maximum of trace(R^T H) over proper
// rotations.  Both are what Horn's quaternion method yields directly: the top eigenpair
// of a symmetric 4x4 matrix built from H (eigenvalue = that trace, eigenvector = the
// rotation as a unit quaternion).  It is solved here by cyclic Jacobi in float64, which
// has no branch on the sign of a determinant and no SVD sign ambiguity.
// The reference evaluates in float32 (numpy / torch on float32 arrays); results agree
// to float32 rounding (tests/test_gpu_metrics.py, golden tests/golden/loss.npz).
#include <algorithm>
#include <hip/hip_runtime.h>

#include "kernels.h"

#pragma clang fp contract(off)

namespace vp3d {
namespace {

constexpr int kMThreads = 128;

// Cyclic Jacobi eigen-decomposition of a symmetric 4x4 matrix: A is overwritten by a
// diagonal matrix of eigenvalues, V (initially identity) collects the eigenvectors
// as columns.  Six sweeps take a well-conditioned 4x4 to double precision.
__device__ void jacobi4(double (&A)[4][4], double (&V)[4][4]) {
    for (int sweep = 0; sweep < 8; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < 4; ++p)
            for (int q = p + 1; q < 4; ++q) off += A[p][q] * A[p][q];
        if (off < 1e-300) break;
        for (int p = 0; p < 3; ++p)
            for (int q = p + 1; q < 4; ++q) {
                const double apq = A[p][q];
                if (fabs(apq) < 1e-300) continue;
                const double theta = (A[q][q] - A[p][p]) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0);
                const double s = t * c;
                for (int k = 0; k < 4; ++k) {  // A <- A J (columns p, q)
                    const double akp = A[k][p], akq = A[k][q];
                    A[k][p] = c * akp - s * akq;
                    A[k][q] = s * akp + c * akq;
                }
                for (int k = 0; k < 4; ++k) {  // A <- J^T A (rows p, q)
                    const double apk = A[p][k], aqk = A[q][k];
                    A[p][k] = c * apk - s * aqk;
                    A[q][k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 4; ++k) {
                    const double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - s * vkq;
                    V[k][q] = s * vkp + c * vkq;
                }
            }
    }
}

__device__ __forceinline__ double norm3(double x, double y, double z) { return sqrt(x * x + y * y + z * z); }

__global__ void pose_metrics_kernel(const float* __restrict__ pred, const float* __restrict__ tgt,
                                    int64_t n_frames, int J, double* __restrict__ acc) {
    double e_mpjpe = 0.0, e_p = 0.0, e_n = 0.0, e_v = 0.0;
    for (int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; f < n_frames;
         f += (int64_t)gridDim.x * blockDim.x) {
        const float* P = pred + f * J * 3;
        const float* T = tgt + f * J * 3;
        // means, Protocol #1, the N-MPJPE scale terms (loss.py:77-78: sums over xyz, means over joints)
        double muX[3] = {0, 0, 0}, muY[3] = {0, 0, 0};
        double pp = 0.0, tp = 0.0;
        for (int j = 0; j < J; ++j) {
            double p[3], t[3];
            for (int c = 0; c < 3; ++c) {
                p[c] = P[3 * j + c];
                t[c] = T[3 * j + c];
                muX[c] += t[c];
                muY[c] += p[c];
            }
            pp += p[0] * p[0] + p[1] * p[1] + p[2] * p[2];
            tp += t[0] * p[0] + t[1] * p[1] + t[2] * p[2];
            e_mpjpe += norm3(p[0] - t[0], p[1] - t[1], p[2] - t[2]);
        }
        for (int c = 0; c < 3; ++c) {
            muX[c] /= J;
            muY[c] /= J;
        }
        const double scale = (tp / J) / (pp / J);
        // centred norms and the cross-covariance S_ab = sum_j y0_a x0_b (y: prediction)
        double nx = 0.0, ny = 0.0, S[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
        for (int j = 0; j < J; ++j) {
            double x0[3], y0[3];
            for (int c = 0; c < 3; ++c) {
                x0[c] = T[3 * j + c] - muX[c];
                y0[c] = P[3 * j + c] - muY[c];
            }
            nx += x0[0] * x0[0] + x0[1] * x0[1] + x0[2] * x0[2];
            ny += y0[0] * y0[0] + y0[1] * y0[1] + y0[2] * y0[2];
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) S[a][b] += y0[a] * x0[b];
        }
        nx = sqrt(nx);
        ny = sqrt(ny);
        const double inv = 1.0 / (nx * ny);  // both point sets divided by their norms
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) S[a][b] *= inv;
        // Horn's symmetric matrix; its top eigenpair is (max trace, rotation quaternion)
        double N4[4][4] = {
            {S[0][0] + S[1][1] + S[2][2], S[1][2] - S[2][1], S[2][0] - S[0][2], S[0][1] - S[1][0]},
            {S[1][2] - S[2][1], S[0][0] - S[1][1] - S[2][2], S[0][1] + S[1][0], S[2][0] + S[0][2]},
            {S[2][0] - S[0][2], S[0][1] + S[1][0], -S[0][0] + S[1][1] - S[2][2], S[1][2] + S[2][1]},
            {S[0][1] - S[1][0], S[2][0] + S[0][2], S[1][2] + S[2][1], -S[0][0] - S[1][1] + S[2][2]}};
        double V[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
        jacobi4(N4, V);
        int k = 0;
        for (int i = 1; i < 4; ++i)
            if (N4[i][i] > N4[k][k]) k = i;
        const double tr = N4[k][k];
        double q0 = V[0][k], qx = V[1][k], qy = V[2][k], qz = V[3][k];
        const double qn = 1.0 / sqrt(q0 * q0 + qx * qx + qy * qy + qz * qz);
        q0 *= qn;
        qx *= qn;
        qy *= qn;
        qz *= qn;
        // Q rotates prediction (column) vectors onto the target; the reference's row-vector
        // R (predicted @ R) is Q^T
        const double Q[3][3] = {
            {1 - 2 * (qy * qy + qz * qz), 2 * (qx * qy - q0 * qz), 2 * (qx * qz + q0 * qy)},
            {2 * (qx * qy + q0 * qz), 1 - 2 * (qx * qx + qz * qz), 2 * (qy * qz - q0 * qx)},
            {2 * (qx * qz - q0 * qy), 2 * (qy * qz + q0 * qx), 1 - 2 * (qx * qx + qy * qy)}};
        const double a = tr * nx / ny;  // loss.py:61
        double tv[3];                   // loss.py:62: muX - a * muY R
        for (int r = 0; r < 3; ++r) tv[r] = muX[r] - a * (Q[r][0] * muY[0] + Q[r][1] * muY[1] + Q[r][2] * muY[2]);
        for (int j = 0; j < J; ++j) {
            double p[3], t[3];
            for (int c = 0; c < 3; ++c) {
                p[c] = P[3 * j + c];
                t[c] = T[3 * j + c];
            }
            double d[3];
            for (int r = 0; r < 3; ++r) d[r] = a * (Q[r][0] * p[0] + Q[r][1] * p[1] + Q[r][2] * p[2]) + tv[r] - t[r];
            e_p += norm3(d[0], d[1], d[2]);
            e_n += norm3(scale * p[0] - t[0], scale * p[1] - t[1], scale * p[2] - t[2]);
            if (f > 0) {
                const float* Pp = P - J * 3;
                const float* Tp = T - J * 3;
                double v[3];
                for (int c = 0; c < 3; ++c)
                    v[c] = ((double)p[c] - Pp[3 * j + c]) - ((double)t[c] - Tp[3 * j + c]);
                e_v += norm3(v[0], v[1], v[2]);
            }
        }
    }
    double vals[4] = {e_mpjpe, e_p, e_n, e_v};
    __shared__ double part[4][kMThreads / 64];
    for (int i = 0; i < 4; ++i) {
        double s = vals[i];
        for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
        if ((threadIdx.x & 63) == 0) part[i][threadIdx.x >> 6] = s;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        double t = 0.0;
        for (int w = 0; w < kMThreads / 64; ++w) t += part[threadIdx.x][w];
        atomicAdd(acc + threadIdx.x, t);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        atomicAdd(acc + 4, (double)n_frames * J);
        atomicAdd(acc + 5, (double)(n_frames > 0 ? n_frames - 1 : 0) * J);
    }
}

}  // namespace

hipError_t launch_pose_metrics(const float* pred, const float* target, int64_t n_frames, int J, double* acc,
                               hipStream_t s) {
    if (n_frames <= 0) return hipSuccess;
    int64_t blocks = (n_frames + kMThreads - 1) / kMThreads;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(pose_metrics_kernel, dim3((unsigned)blocks), dim3(kMThreads), 0, s, pred, target, n_frames,
                       J, acc);
    return hipGetLastError();
}

}  // namespace vp3d

namespace vp3d {
namespace {
// any non-finite value of y[0, n) -> OR `bit` into the (host-mapped) fault word; one grid-stride
// pass (float4 loads when y is 16-byte aligned, else element-wise), the flag touched only by a
// wave that found one
template <bool VEC>
__global__ void nonfinite_check_kernel(const float* __restrict__ y, int64_t n, unsigned* flag, unsigned bit) {
    bool bad = false;
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    const int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if constexpr (VEC) {
        const float4* y4 = reinterpret_cast<const float4*>(y);
        const int64_t n4 = n / 4;
        for (int64_t i = i0; i < n4; i += step) {
            const float4 v = y4[i];
            bad |= !__builtin_isfinite(v.x) || !__builtin_isfinite(v.y) || !__builtin_isfinite(v.z) ||
                   !__builtin_isfinite(v.w);
        }
        if (i0 < n - 4 * n4) bad |= !__builtin_isfinite(y[4 * n4 + i0]);
    } else {
        for (int64_t i = i0; i < n; i += step) bad |= !__builtin_isfinite(y[i]);
    }
    if (__any(bad) && (threadIdx.x & 63) == 0)
        __hip_atomic_fetch_or(flag, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace

hipError_t launch_nonfinite_check(const float* y, int64_t n, unsigned* flag, unsigned bit, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const bool vec = (reinterpret_cast<uintptr_t>(y) & 15) == 0;
    const int64_t per = vec ? (n + 3) / 4 : n;
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((per + 255) / 256, 1024));
    if (vec)
        hipLaunchKernelGGL(nonfinite_check_kernel<true>, dim3(blocks), dim3(256), 0, s, y, n, flag, bit);
    else
        hipLaunchKernelGGL(nonfinite_check_kernel<false>, dim3(blocks), dim3(256), 0, s, y, n, flag, bit);
    return hipGetLastError();
}
}  // namespace vp3d
