// Causal streaming step as ONE persistent launch per batch of frames (BASELINE config 5).
//
// Model: the causal dilated TemporalModel (reference common/models/TemporalModel.py:79-138,
// causal=True: block b's residual is the newest frame of its input, :132; output t of a
// k-conv reads its input at times t - 2d, t - d, t, clamped at 0 — the 2*pad copies of
// frame 0 the reference's UnchunkedGenerator puts in front of a causal sequence,
// generators.py:193-198).
//
// Layout: every workgroup (one per CU) owns CPW output channels of EVERY layer and keeps
// their 16-bit weights resident in LDS for the whole launch (at 1024 channels, CPW = 4:
// 4 x (102 + 4 x (3072 + 1024) + 1024) halves = 137 KB), so a step moves no weights.
// Per step the layers hand their output vectors to every CU through 8-byte {tag, value}
// granules (write-through agent-scope stores, relaxed agent-scope polls: the R2 hand-off
// of cdna_hip_programming.md Guideline 16; the tag is the step index within the launch
// + 1, every granule zeroed by a memset before each launch; one buffer per edge and step
// parity, so a fast producer never overwrites a granule a slow consumer still waits for).
//
// The k-convs are split by tap so that only the newest tap is on the step's critical
// path: when x(t) arrives, W2 x(t) completes output t (partial[t] + W2 x(t)), and
// W1 x(t) / W0 x(t) are added to the partial sums of outputs t + d / t + 2d, kept in a
// per-CU ring of 2d + 1 slots.  At t = 0 the clamped taps make output 0 = (W0+W1+W2) x(0),
// outputs 1..d start from (W0 + W1) x(0) and outputs d+1..2d from W0 x(0).
//
// Per step: 9 hand-off edges (expand out, then per block the k-conv and 1x1 outputs);
// the shrink runs on the few CUs that own its 51 rows.  Every spin is bounded (~0.25 s
// of the 100 MHz clock); a timeout sets the sticky error word and every wave leaves.
#include <stdint.h>

#include "kernels.h"

namespace vp3d {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;

constexpr int kThreads = 256;
constexpr int kWaves = 4;
constexpr int kLds = 156 * 1024;  // one workgroup per CU

__device__ __forceinline__ float wave_sum(float s) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    return s;
}

// dot of 8 16-bit weights (one 16-byte LDS word) with 8 floats
template <typename WT>
__device__ __forceinline__ float dot8(u32x4 w, const float* x, float s) {
    typedef WT wt8 __attribute__((ext_vector_type(8)));
    const wt8 v = __builtin_bit_cast(wt8, w);
    const float4 a = *(const float4*)x;
    const float4 b = *(const float4*)(x + 4);
    s = __builtin_fmaf((float)v[0], a.x, s);
    s = __builtin_fmaf((float)v[1], a.y, s);
    s = __builtin_fmaf((float)v[2], a.z, s);
    s = __builtin_fmaf((float)v[3], a.w, s);
    s = __builtin_fmaf((float)v[4], b.x, s);
    s = __builtin_fmaf((float)v[5], b.y, s);
    s = __builtin_fmaf((float)v[6], b.z, s);
    s = __builtin_fmaf((float)v[7], b.w, s);
    return s;
}

// lane-partial dot of one weight row segment (n 16-bit elements, n % 8 == 0) with x (LDS)
template <typename WT>
__device__ __forceinline__ float row_dot(const WT* w, const float* x, int n, int lane) {
    float s = 0.f;
    for (int k = lane * 8; k < n; k += 512) s = dot8<WT>(*(const u32x4*)(w + k), x + k, s);
    return s;
}

__device__ __forceinline__ void publish(gu64* g, unsigned epoch, float v) {
    const unsigned long long x = ((unsigned long long)epoch << 32) | __float_as_uint(v);
    __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

// Sweep the C granules of one edge into LDS: every thread owns granules tid + j*256,
// polls the ones still missing (four loads in flight per pass), and returns true once
// every tag matched; false on timeout (sets the sticky error word) or when another
// wave of the workgroup aborted.
__device__ __forceinline__ bool sweep(gu64* g, int C, unsigned epoch, float* x, volatile int* abort_flag,
                                      const StreamFault& f, int tid) {
    const unsigned long long start = __builtin_amdgcn_s_memrealtime();
    for (int i0 = tid; i0 < C; i0 += 4 * kThreads) {
        unsigned pending = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (i0 + j * kThreads < C) pending |= 1u << j;
        for (;;) {
            unsigned long long v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int i = i0 + j * kThreads < C ? i0 + j * kThreads : C - 1;
                v[j] = __hip_atomic_load(g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (((pending >> j) & 1u) && (unsigned)(v[j] >> 32) == epoch) {
                    x[i0 + j * kThreads] = __uint_as_float((unsigned)v[j]);
                    pending &= ~(1u << j);
                }
            if (!pending) break;
            if (*abort_flag) return false;
            if (__builtin_amdgcn_s_memrealtime() - start > f.spin_ticks) {
                *abort_flag = 1;
                __hip_atomic_store((gu32*)f.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (f.err_host) __hip_atomic_store(f.err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return false;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    return true;
}

template <typename WT>
__global__ __launch_bounds__(kThreads, 1) void stream_persist_kernel(StreamPersistParams p) {
    __shared__ __attribute__((aligned(16))) char smem[kLds];
    __shared__ int abort_flag;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wg = blockIdx.x;
    const int C = p.C, CPW = p.CPW, nb = p.nb, cin0 = p.cin0;
    const int c0 = wg * CPW;
    // a stream that timed out stays failed until vp3d_stream_reset: no-op launches, so the
    // frame position and the partial-sum rings never drift out of step
    if (__hip_atomic_load(p.fault.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    if (tid == 0) abort_flag = 0;

    // ---- LDS carve (byte offsets precomputed on the host, all 16-byte aligned) ----
    const WT* w_l[kStreamMaxLayers];
    for (int l = 0; l < p.nl; ++l) w_l[l] = (const WT*)(smem + p.w_off[l]);
    float* xbuf = (float*)(smem + p.x_off);       // swept input vector, C floats
    float* xin = (float*)(smem + p.xin_off);      // expand input: 3 frames x cin0 (+ pad)
    float* hist = (float*)(smem + p.hist_off);    // frames t-1, t-2
    float* part = (float*)(smem + p.part_off);    // partial-sum rings, CPW per slot
    float* scl = (float*)(smem + p.ss_off);       // [layer][CPW] scale, then shift

    // ---- weights of this workgroup's rows into LDS (zero rows past N) ----
    for (int l = 0; l < p.nl; ++l) {
        const int rows = CPW, Kp = p.Kp[l];
        const int r0 = l == p.nl - 1 ? wg * CPW : c0;  // shrink rows: outputs wg*CPW..
        const int kv = Kp / 8;
        for (int i = tid; i < rows * kv; i += kThreads) {
            const int r = i / kv, k = (i - r * kv) * 8;
            const int n = r0 + r;
            u32x4 v = {0u, 0u, 0u, 0u};
            if (n < p.N[l]) v = *(const u32x4*)((const WT*)p.W[l] + (int64_t)n * Kp + k);
            *(u32x4*)((WT*)(smem + p.w_off[l]) + r * Kp + k) = v;
        }
        for (int r = tid; r < CPW; r += kThreads) {
            const int n = r0 + r;
            scl[(2 * l) * CPW + r] = n < p.N[l] ? p.scale[l][n] : 0.f;
            scl[(2 * l + 1) * CPW + r] = n < p.N[l] ? p.shift[l][n] : 0.f;
        }
    }
    // ---- persistent per-workgroup state: partial rings + frame history ----
    float* gstate = p.state + (int64_t)wg * p.state_floats;
    for (int i = tid; i < p.part_floats; i += kThreads) part[i] = gstate[i];
    for (int i = tid; i < 2 * cin0; i += kThreads) hist[i] = gstate[p.part_floats + i];
    const int t0 = *p.frames_seen;
    __syncthreads();

    const int nsh = (p.N[p.nl - 1] + CPW - 1) / CPW;  // workgroups that own shrink rows
    for (int s = 0; s < p.steps; ++s) {
        const int t = t0 + s;
        const unsigned epoch = (unsigned)s + 1u;
        const int par = s & 1;
        auto edge = [&](int e) { return (gu64*)p.gran + ((int64_t)(e * 2 + par)) * C; };

        // ---- expand: frames t-2, t-1, t (clamped at 0) -> x1(t), own channels ----
        const float* fr = p.frames + (int64_t)(t & (p.queue - 1)) * cin0;
        for (int i = tid; i < cin0; i += kThreads) {
            const float v = fr[i];
            const float h1 = t == 0 ? v : hist[i];             // frame t-1
            const float h2 = t <= 1 ? (t == 0 ? v : h1) : hist[cin0 + i];  // frame t-2
            xin[i] = h2;
            xin[cin0 + i] = h1;
            xin[2 * cin0 + i] = v;
        }
        for (int i = 3 * cin0 + tid; i < p.Kp[0]; i += kThreads) xin[i] = 0.f;
        __syncthreads();
        // history for the next step (every wave has read it: the barrier above)
        for (int i = tid; i < cin0; i += kThreads) {
            hist[cin0 + i] = xin[cin0 + i];
            hist[i] = xin[2 * cin0 + i];
        }
        float xres = 0.f;  // this wave's channel of the current block input (the residual)
        if (wid < CPW) {
            float sacc = row_dot<WT>(w_l[0] + wid * p.Kp[0], xin, p.Kp[0], lane);
            sacc = wave_sum(sacc);
            float y = sacc * scl[0 * CPW + wid] + scl[1 * CPW + wid];
            y = y > 0.f ? y : 0.f;
            if (lane == 0) publish(edge(0) + c0 + wid, epoch, y);
        }

        // ---- residual blocks ----
        int ring_base = 0;
        for (int b = 1; b <= nb; ++b) {
            const int lk = 2 * b - 1, lp = 2 * b;
            const int d = p.dil[b], R = p.ring[b];
            // x_b(t) from every CU
            if (!sweep(edge(2 * b - 2), C, epoch, xbuf, &abort_flag, p.fault, tid)) abort_flag = 1;
            __syncthreads();
            if (abort_flag) return;
            if (wid < CPW) {
                const WT* w = w_l[lk] + wid * p.Kp[lk];
                const int taps = p.taps[b];
                xres = xbuf[c0 + wid];
                // newest tap first: it completes output t
                const float vn = wave_sum(row_dot<WT>(w + (taps - 1) * C, xbuf, C, lane));
                float* pr = part + (ring_base * CPW);
                float out;
                if (t == 0) {
                    // every tap reads x(0); outputs 1 .. (taps-1) d start from the taps that
                    // still reach before the stream start
                    float vk[kStreamMaxTaps];
                    out = 0.f;
                    for (int k = 0; k < taps - 1; ++k) {
                        vk[k] = wave_sum(row_dot<WT>(w + k * C, xbuf, C, lane));
                        out += vk[k];
                    }
                    out += vn;
                    float hv = out * scl[(2 * lk) * CPW + wid] + scl[(2 * lk + 1) * CPW + wid];
                    hv = hv > 0.f ? hv : 0.f;
                    if (lane == 0) {
                        publish(edge(2 * b - 1) + c0 + wid, epoch, hv);
                        for (int q = 0; q < R; ++q) pr[q * CPW + wid] = 0.f;
                        for (int tt = 1; tt <= (taps - 1) * d; ++tt) {
                            float acc = 0.f;
                            for (int k = 0; k < taps - 1; ++k)
                                if ((taps - 1 - k) * d >= tt) acc += vk[k];
                            pr[(tt & (R - 1)) * CPW + wid] = acc;
                        }
                    }
                } else {
                    out = pr[(t & (R - 1)) * CPW + wid] + vn;
                    float hv = out * scl[(2 * lk) * CPW + wid] + scl[(2 * lk + 1) * CPW + wid];
                    hv = hv > 0.f ? hv : 0.f;
                    if (lane == 0) publish(edge(2 * b - 1) + c0 + wid, epoch, hv);
                    // the older taps of this x(t) feed outputs t + (taps-1-k) d (off the critical path)
                    if (lane == 0) pr[(t & (R - 1)) * CPW + wid] = 0.f;
                    for (int k = taps - 2; k >= 0; --k) {
                        const float v = wave_sum(row_dot<WT>(w + k * C, xbuf, C, lane));
                        if (lane == 0) pr[((t + (taps - 1 - k) * d) & (R - 1)) * CPW + wid] += v;
                    }
                }
            }
            ring_base += R;
            __syncthreads();  // xbuf is overwritten by the next sweep
            // h_b(t) from every CU
            if (!sweep(edge(2 * b - 1), C, epoch, xbuf, &abort_flag, p.fault, tid)) abort_flag = 1;
            __syncthreads();
            if (abort_flag) return;
            if (wid < CPW) {
                const float v = wave_sum(row_dot<WT>(w_l[lp] + wid * p.Kp[lp], xbuf, C, lane));
                float y = v * scl[(2 * lp) * CPW + wid] + scl[(2 * lp + 1) * CPW + wid];
                y = y > 0.f ? y : 0.f;
                y += xres;
                if (lane == 0) publish(edge(2 * b) + c0 + wid, epoch, y);
            }
            __syncthreads();
        }
        // ---- shrink on the workgroups that own its rows ----
        if (wg < nsh) {
            if (!sweep(edge(2 * nb), C, epoch, xbuf, &abort_flag, p.fault, tid)) abort_flag = 1;
            __syncthreads();
            if (abort_flag) return;
            const int ls = p.nl - 1;
            const int o = wg * CPW + wid;
            if (wid < CPW && o < p.N[ls]) {
                const float v = wave_sum(row_dot<WT>(w_l[ls] + wid * p.Kp[ls], xbuf, C, lane));
                if (lane == 0)
                    p.poses[(int64_t)(t & (p.queue - 1)) * p.N[ls] + o] =
                        v * scl[(2 * ls) * CPW + wid] + scl[(2 * ls + 1) * CPW + wid];
            }
            __syncthreads();
        }
    }
    // ---- save the per-workgroup state; advance the stream position ----
    __syncthreads();
    for (int i = tid; i < p.part_floats; i += kThreads) gstate[i] = part[i];
    for (int i = tid; i < 2 * cin0; i += kThreads) gstate[p.part_floats + i] = hist[i];
    if (wg == 0 && tid == 0) *p.frames_seen = t0 + p.steps;
}

int stream_persist_lds_bytes() { return kLds; }

hipError_t launch_stream_persist(const StreamPersistParams& p, Act wtype, hipStream_t s) {
    if (wtype == Act::F16)
        hipLaunchKernelGGL(stream_persist_kernel<_Float16>, dim3(p.G), dim3(kThreads), 0, s, p);
    else if (wtype == Act::BF16)
        hipLaunchKernelGGL(stream_persist_kernel<__bf16>, dim3(p.G), dim3(kThreads), 0, s, p);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace vp3d
