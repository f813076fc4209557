// Causal streaming step: one new 2D frame in, one 3D pose out (BASELINE config 5).
//
// The causal dilated TemporalModel (reference common/models/TemporalModel.py:79-138
// with causal=True; causal_shift = pad, so block i's residual is the NEWEST frame
// of its input, :132) evaluated one frame at a time.  Every convolution becomes a
// GEMV over the layer's taps, read from per-layer ring buffers of past activations:
//
//   layer input x_i (C floats per frame) kept for 2*d_i + 1 frames (ring of R_i = 2^k)
//   k-conv(t)  = sum_k W_k x_i[t - (w-1-k) d_i]          (TemporalModel.py:134)
//   x_{i+1}(t) = x_i[t] + relu(bn(W_1x1 relu(bn(k-conv(t)))))  (:135)
//
// Stream start: the reference edge-pads a causal sequence with 2*pad copies of
// frame 0 (generators.py:193-198 with causal_shift = pad).  Every activation whose
// aligned time is <= 0 therefore equals the one at time 0, so a tap that reaches
// before the stream start reads time 0 — exact equivalence, no warm-up frames.
//
// The stream position lives in device memory (frames_seen), read by every kernel
// and advanced by the last one, so the whole step is replayable from a hipGraph
// with fixed kernel arguments.
//
// Each kernel is weight-streaming (1 FLOP per weight byte at fp16): the GEMV
// stages the layer's input vector in LDS and every wave streams one whole weight
// row with all of its 16-byte loads in flight at once.  Frames come from a device
// queue indexed by the stream position and poses go to a ring, so one graph can
// hold several consecutive steps with no host work between them.
#include "kernels.h"

namespace vp3d {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kMaxK = 4096;  // per-step input vector (taps * Cin) staged in LDS

template <typename WT>
__device__ __forceinline__ float wdot8(const u32x4 w, const float* v) {
    typedef WT wt8 __attribute__((ext_vector_type(8)));
    const wt8 x = __builtin_bit_cast(wt8, w);
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) s = __builtin_fmaf((float)x[e], v[e], s);
    return s;
}

template <>
__device__ __forceinline__ float wdot8<float>(const u32x4 w, const float* v) {
    (void)w;
    (void)v;
    return 0.f;  // f32 weights use the 4-wide path below
}

__device__ __forceinline__ float wave_sum(float s) {
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    return s;
}

// One streaming GEMV layer.  in: input ring (or plain vector when in_R == 0);
// the expand layer additionally reads the newest frame from the frame queue.
constexpr int kMaxIter = 8;  // Kp <= 4096 halves: 8 x 512 fp16 elements per row

template <typename WT>
__global__ __launch_bounds__(256) void stream_gemv(StreamLayerParams q) {
    __shared__ __attribute__((aligned(16))) float v[kMaxK];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int n = blockIdx.x * (blockDim.x >> 6) + (tid >> 6);

    // 1. the weight row does not depend on the stream position: put all of its
    //    16-byte loads in flight first, so their latency overlaps the staging below
    u32x4 w[kMaxIter];
    if constexpr (sizeof(WT) == 2) {
        if (n < q.N) {
            const WT* wr = (const WT*)q.W + (int64_t)n * q.Kp + lane * 8;
#pragma unroll
            for (int it = 0; it < kMaxIter; ++it)
                if (it * 512 + lane * 8 < q.Kp) w[it] = *(const u32x4*)(wr + it * 512);
        }
    }

    // per-row epilogue operands do not depend on the stream position either
    float sc = 0.f, sh = 0.f;
    if (n < q.N && lane == 0) {
        sc = q.scale[n];
        sh = q.shift[n];
    }

    // 2. stage the input vector: tap k reads stream time t - (taps-1-k)*dil, clamped at 0.
    //    A plain (non-ring) input does not depend on t: its loads go out before t arrives,
    //    so the two memory round trips overlap instead of chaining.
    const bool plain = !q.in_R && !q.in_frame;
    if (plain)
        for (int kk = tid; kk < q.taps * q.cin; kk += blockDim.x) v[kk] = q.in[kk % q.cin];
    const int t = *q.frames_seen;
    // the residual row of this step (lane 0 of each wave), loaded ahead of the dot product
    float rv = 0.f;
    if (q.res && n < q.N && lane == 0) rv = q.res[(int64_t)(q.res_R ? (t & (q.res_R - 1)) : 0) * q.N + n];
    const float* frame = q.in_frame ? q.in_frame + (int64_t)(t & (q.in_frame_R - 1)) * q.cin : nullptr;
    if (!plain) {
        for (int tap = 0; tap < q.taps; ++tap) {
            int tt = t - (q.taps - 1 - tap) * q.dil;
            tt = tt < 0 ? 0 : tt;
            const float* src = (frame && tt == t) ? frame
                               : (q.in_R ? q.in + (int64_t)(tt & (q.in_R - 1)) * q.cin : q.in);
            for (int c = tid; c < q.cin; c += blockDim.x) v[tap * q.cin + c] = src[c];
        }
    }
    for (int kk = q.K + tid; kk < q.Kp; kk += blockDim.x) v[kk] = 0.f;
    // the expand layer also appends the new frame to its input ring (slot of time t;
    // this step's other taps read older slots, so no workgroup races with it)
    if (frame && q.in_ring_w && blockIdx.x == 0)
        for (int c = tid; c < q.cin; c += blockDim.x)
            q.in_ring_w[(int64_t)(t & (q.in_R - 1)) * q.cin + c] = frame[c];
    __syncthreads();

    // 3. dot products
    if (n < q.N) {
        float s = 0.f;
        if constexpr (sizeof(WT) == 2) {
#pragma unroll
            for (int it = 0; it < kMaxIter; ++it)
                if (it * 512 + lane * 8 < q.Kp) s += wdot8<WT>(w[it], &v[it * 512 + lane * 8]);
        } else {
            const float* wr = (const float*)q.W + (int64_t)n * q.Kp + lane * 4;
            for (int k0 = 0; k0 < q.Kp; k0 += 256 * 4) {
                float4 w4[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (k0 + u * 256 + lane * 4 < q.Kp) w4[u] = *(const float4*)(wr + k0 + u * 256);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = k0 + u * 256 + lane * 4;
                    if (k < q.Kp) {
                        s = __builtin_fmaf(w4[u].x, v[k], s);
                        s = __builtin_fmaf(w4[u].y, v[k + 1], s);
                        s = __builtin_fmaf(w4[u].z, v[k + 2], s);
                        s = __builtin_fmaf(w4[u].w, v[k + 3], s);
                    }
                }
            }
        }
        s = wave_sum(s);
        if (lane == 0) {
            float y = s * sc + sh;
            if (q.relu) y = y > 0.f ? y : 0.f;
            if (q.res) y += rv;
            const int64_t o = q.out_R ? (int64_t)(t & (q.out_R - 1)) * q.N + n : n;
            q.out[o] = y;
        }
    }
    if (q.advance) {
        // last layer of the step: the last workgroup to finish advances the stream
        // position (every workgroup read t before its arrival is counted)
        __syncthreads();
        if (tid == 0) {
            const unsigned done = __hip_atomic_fetch_add(q.done_counter, 1u, __ATOMIC_ACQ_REL,
                                                         __HIP_MEMORY_SCOPE_AGENT);
            if (done == gridDim.x - 1) {
                *q.done_counter = 0u;
                __hip_atomic_store(q.frames_seen, t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

}  // namespace

hipError_t launch_stream_gemv(const StreamLayerParams& q, Act wtype, hipStream_t s) {
    if (q.Kp > kMaxK) return hipErrorInvalidValue;
    const int nwaves = 4;  // one output row per wave
    const int grid = (q.N + nwaves - 1) / nwaves;
    const dim3 block(64 * nwaves);
    if (wtype == Act::F32)
        hipLaunchKernelGGL(stream_gemv<float>, dim3(grid), block, 0, s, q);
    else if (wtype == Act::F16)
        hipLaunchKernelGGL(stream_gemv<_Float16>, dim3(grid), block, 0, s, q);
    else
        hipLaunchKernelGGL(stream_gemv<__bf16>, dim3(grid), block, 0, s, q);
    return hipGetLastError();
}

}  // namespace vp3d
