// Causal streaming step as ONE layer-pipelined persistent launch per batch of frames
// (BASELINE config 5, 16-bit weights).
//
// Model: the causal dilated TemporalModel (reference common/models/TemporalModel.py:79-138,
// causal=True: block b's residual is the newest frame of its input, :132; output t of a
// k-conv reads its input at times t - 2d, t - d, t, clamped at 0 -- the 2*pad copies of
// frame 0 that UnchunkedGenerator puts in front of a causal sequence, generators.py:193-198).
//
// Why another form (stream_persist.hip spreads every layer over all 256 CUs): there, each
// of the 9 layer outputs of a step is an all-to-all edge read by all 256 CUs, ~2.5 us each
// (MI355X_MICROARCH.md "allgather"), and a step cannot start before the previous one has
// left the last layer.  Here every workgroup (one per CU) owns ONE layer -- its "role":
// expand, block b's k-conv, block b's 1x1 conv, or the shrink -- and a slice of that
// layer's output channels, with the slice's 16-bit weights resident in VGPRs for the whole
// launch.  A layer output is then read only by the next layer's group (46 / 16 CUs at 1024
// channels instead of 256), and the groups form a pipeline over the frames of the batch:
// while block 4 works on frame t, block 1 already works on frame t + 3.  Results are the
// same as one frame at a time (no group reads anything a later frame writes).
//
// Hand-off: 8-byte {tag, value} granules (R2 of cdna_hip_programming.md Guideline 16:
// write-through agent-scope stores, relaxed agent-scope polls); tag = absolute frame
// index + 1, one granule slot per (frame % queue, edge, channel), so no per-launch zeroing
// (vp3d_stream_reset clears them) and no producer can lap a consumer inside a launch.
//
// Layouts (one wave = 64 lanes):
//   * k-conv / 1x1 / shrink ("k-sliced"): lane L holds elements [L*KS, L*KS + KS) of every
//     weight row the wave owns (KS = C / 64); a channel's dot product is a lane-partial sum
//     reduced across the wave (DPP within 16-lane rows, then the 4 row sums).
//   * expand ("lane per channel"): lane L owns one output channel and its whole weight row
//     (K = 3 * 34 = 102, padded to 128); the 3-frame input vector is an LDS broadcast.
// Weights are held as f32 pairs in VGPRs (16-bit weights widened exactly once at launch; the
// exact-fp32 form, WT = float, loads them as they are -- the same registers either way) and
// every dot product runs on v_pk_fma_f32 with f32 activations, so the fp32 form differs from
// the reference only by the order of its f32 sums.
//
// Block b's k-conv is split by tap (as in stream_persist.hip): the newest tap completes
// output t; the older taps' products of x(t) go into a wave-private ring of partial sums
// for outputs t + d and t + 2d, off the critical path.  Every spin is bounded (~0.25 s of
// the 100 MHz clock); a timeout sets the sticky error word and the workgroup leaves.
#include <stdint.h>

#include "kernels.h"

namespace vp3d {
namespace {

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;

constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;

// 16-bit weight halves of a packed u32 -> f32 (exact)
template <typename WT>
__device__ __forceinline__ float lo16(uint32_t w) {
    return (float)__builtin_bit_cast(WT, (unsigned short)(w & 0xffffu));
}
template <typename WT>
__device__ __forceinline__ float hi16(uint32_t w) {
    return (float)__builtin_bit_cast(WT, (unsigned short)(w >> 16));
}

typedef float f2 __attribute__((ext_vector_type(2)));

// 16-bit weight pair -> two f32 (exact), converted once when the weights are loaded: the
// dot products then run as v_pk_fma_f32 (two FMAs per instruction) on f32 pairs instead of a
// convert + FMA per element every frame
template <typename WT>
__device__ __forceinline__ f2 widen2(uint32_t w) {
    return f2{lo16<WT>(w), hi16<WT>(w)};
}

// weight pair i of a row (elements 2i, 2i + 1) as f32: a widened 16-bit pair, or two f32 as stored
template <typename WT>
__device__ __forceinline__ f2 wpair(const WT* row, int i) {
    if constexpr (sizeof(WT) == 4) {
        const float2 v = *(const float2*)(row + 2 * i);
        return f2{v.x, v.y};
    } else {
        return widen2<WT>(((const uint32_t*)row)[i]);
    }
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// Lane-partial sums of CW <= 8 rows -> row totals, as a reduce-scatter over the wave: each
// exchange step halves the rows a lane still carries (v_permlane32_swap: lanes 0-31 keep the
// first half of the rows, 32-63 the second; v_permlane16_swap: the same between even and
// odd 16-lane rows; for 8 rows a DPP rotate by 8 inside the 16-lane row), then the lanes that
// share a row add up (DPP xor 1, xor 2, half mirror[, mirror]).  Lane l returns the total of
// row l >> 3 (CW > 4) or l >> 4 (CW <= 4; rows past CW are zero).  About 18 instructions for
// 8 rows instead of 8 full-wave reductions and the moves that put row j's sum into lane j.
template <int CW>
__device__ __forceinline__ float rows_sum(const float (&v)[CW], int lane) {
    constexpr int P = CW <= 4 ? 4 : 8;
    float s[P];
#pragma unroll
    for (int j = 0; j < P; ++j) s[j] = j < CW ? v[j] : 0.f;
#pragma unroll
    for (int k = 0; k < P / 2; ++k) {
        float x = s[k], y = s[k + P / 2];
        // x, y were just written by VALU -> 2 wait states (inline asm: see gemm_common.h)
        asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
        s[k] = x + y;  // lanes 0-31: row k, lanes 32-63: row k + P/2
    }
#pragma unroll
    for (int k = 0; k < P / 4; ++k) {
        float x = s[k], y = s[k + P / 4];
        asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
        s[k] = x + y;  // even 16-lane rows: row k (+ P/2), odd: row k + P/4 (+ P/2)
    }
    float r;
    if constexpr (P == 8) {
        const float a = s[0] + dpp<0x128>(s[0]), b = s[1] + dpp<0x128>(s[1]);  // row_ror:8 = xor 8
        r = (lane & 8) ? b : a;
    } else {
        r = s[0];
    }
    r += dpp<0xB1>(r);   // xor 1
    r += dpp<0x4E>(r);   // xor 2
    r += dpp<0x141>(r);  // half mirror: the other quad of the 8 lanes
    if constexpr (P == 4) r += dpp<0x140>(r);  // mirror: the other 8 lanes of the 16
    return r;
}

__device__ __forceinline__ void publish(gu64* g, unsigned tag, float v) {
    const unsigned long long x = ((unsigned long long)tag << 32) | __float_as_uint(v);
    __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Granule slice of an edge: element c lives at base + (c0 + c) / 64 * cs + (c0 + c) % 64, i.e.
// 64-granule (512-byte) chunks cs granules apart (cs = 64: contiguous; larger: every chunk
// on its own 4 KB page, so the polls of one edge spread over more memory channels)
struct EdgeRef {
    const gu64* base;
    int c0, cs;
    __device__ __forceinline__ const gu64* at(int c) const { return base + ((c0 + c) >> 6) * cs + ((c0 + c) & 63); }
};

// A sweep split in two so that the next frame's granule loads are in flight while the
// current frame computes: pref_issue loads this thread's granules (tid, tid + kThreads of
// an edge slice of n <= 2 * kThreads), pref_finish checks their tags, re-polls the ones
// still missing (bounded, as sweep) and stores the values into x (LDS).
struct Pref {
    unsigned long long v[2];
};

constexpr unsigned long long kEndCheckTicks = 1000;  // 10 us of the 100 MHz clock

__device__ __forceinline__ void pref_issue(Pref& r, const EdgeRef& e, int n, int tid, unsigned mask = 3u) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
        if (((mask >> j) & 1u) && tid + j * kThreads < n)
            r.v[j] = __hip_atomic_load(e.at(tid + j * kThreads), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool pref_check(const Pref& r, unsigned& pending, unsigned tag, float* x, int tid) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
        if (((pending >> j) & 1u) && (unsigned)(r.v[j] >> 32) == tag) {
            x[tid + j * kThreads] = __uint_as_float((unsigned)r.v[j]);
            pending &= ~(1u << j);
        }
    return pending == 0;
}

__device__ __forceinline__ void poll_pause(int n) {
    for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(1);
}

// true once every granule carried `tag`; false on timeout (sets the fault words) or when
// another wave aborted, or -- serve form -- once the launch ended before frame tag - 1
// (*end < tag: that frame is never produced; *ended is then set).
// One poll of the missing granules in flight, waited for before the next, `pause` x
// s_sleep 1 between polls.  (Two rounds in flight measured slower: 0.5-0.7 us more per
// hand-off, tools/stream_latency.py; and a round still in flight when the function returns
// makes the compiler drain vmcnt before the next reuse of its registers -- which was the
// prefetch of the next frame.)
__device__ bool pref_finish(Pref& r, const EdgeRef& e, int n, unsigned tag, float* x, volatile int* abort_flag,
                            const StreamFault& f, int tid, int pause, unsigned long long limit = 0,
                            const unsigned* end = nullptr, volatile int* ended = nullptr) {
    if (limit == 0) limit = f.spin_ticks;
    unsigned pending = 0;
#pragma unroll
    for (int j = 0; j < 2; ++j)
        if (tid + j * kThreads < n) pending |= 1u << j;
    if (pref_check(r, pending, tag, x, tid)) return true;  // the round issued during the last frame
    const unsigned long long start = __builtin_amdgcn_s_memrealtime();
    // 0: keep polling, 1: aborted / timed out, 2: the launch ended before this frame
    auto give_up = [&]() -> int {
        if (*abort_flag) return 1;
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        // the end word only after a while: its load would otherwise add a round trip to
        // every poll of a frame that is merely in flight
        if (end && now - start > kEndCheckTicks &&
            __hip_atomic_load(end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < tag) {
            *ended = 1;
            return 2;
        }
        if (now - start > limit) {
            *abort_flag = 1;
            __hip_atomic_store((gu32*)f.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (f.err_host) __hip_atomic_store(f.err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return 1;
        }
        return 0;
    };
    for (;;) {
        pref_issue(r, e, n, tid, pending);
        if (pref_check(r, pending, tag, x, tid)) return true;
        if (give_up()) return false;
        poll_pause(pause);
    }
}

// Lane-partial dot products of the wave's CW rows (NT taps each) with the lane's KS input
// elements xl (as KS/2 pairs): s[j] = sum_i w[tap][j][i] . xl[i], even and odd elements in
// the two halves of one v_pk_fma_f32 chain, added at the end.
template <int NT, int CW, int KS>
__device__ __forceinline__ void lane_dots(const f2 (&w)[NT][CW][KS / 2], const f2 (&xl)[KS / 2], int tap,
                                          float (&s)[CW]) {
#pragma unroll
    for (int j = 0; j < CW; ++j) {
        f2 a = f2{0.f, 0.f};
#pragma unroll
        for (int i = 0; i < KS / 2; ++i) a = __builtin_elementwise_fma(w[tap][j][i], xl[i], a);
        s[j] = a.x + a.y;
    }
}

// Row j (< CW) of wave w: contiguous (c_lo + CW w + j: a wave's results are neighbouring
// granules, 8 rows = one 64-byte line written by one store) or strided (c_lo + w + 8 j).
template <int CW>
__device__ __forceinline__ int row_of(int c_lo, int wid, int j, int contig) {
    return contig ? c_lo + CW * wid + j : c_lo + wid + kWaves * j;
}

// Load the wave's rows of one layer into registers: row c = row_of(j), tap
// segment [tap * C + lane * KS, +KS) of the [Np][Kp] 16-bit matrix (rows past c_hi: zero).
template <typename WT, int NT, int CW, int KS>
__device__ __forceinline__ void load_rows(f2 (&w)[NT][CW][KS / 2], const WT* W, int Kp, int C, int c_lo, int c_hi,
                                          int wid, int lane, int taps, int contig) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < CW; ++j) {
            const int c = row_of<CW>(c_lo, wid, j, contig);
#pragma unroll
            for (int i = 0; i < KS / 2; ++i) w[t][j][i] = f2{0.f, 0.f};
            if (c < c_hi && t < taps) {
                const WT* src = W + (int64_t)c * Kp + t * C + lane * KS;
#pragma unroll
                for (int i = 0; i < KS / 2; ++i) w[t][j][i] = wpair<WT>(src, i);
            }
        }
}

template <int KS>
__device__ __forceinline__ void load_x(f2 (&xl)[KS / 2], const float* x, int lane) {
#pragma unroll
    for (int i = 0; i < KS; i += 4) {
        const float4 v = *(const float4*)(x + lane * KS + i);
        xl[i / 2] = f2{v.x, v.y};
        xl[i / 2 + 1] = f2{v.z, v.w};
    }
}

__device__ __forceinline__ void trace_mark(const StreamPipeParams& p, int wg, int s, int k, int tid) {
    // k = 0: thread 0 once the frame's input is complete (slot 0, and the shader clock in
    // slot 9); k = 1: lane 0 of each wave after its first output store (slot 1 + wave; wave 0
    // also the shader clock in slot 10)
    if (p.trace && s < p.trace_frames && (k ? (tid & 63) == 0 : tid == 0)) {
        unsigned long long* e = p.trace + ((int64_t)wg * p.trace_frames + s) * kStreamTraceSlots;
        e[k ? 1 + (tid >> 6) : 0] = __builtin_amdgcn_s_memrealtime();
        if (tid == 0) e[k ? 10 : 9] = __builtin_amdgcn_s_memtime();
    }
}

}  // namespace

// SERVE: the serve form (p.serve; the resident one-frame-in-flight launch) as its own
// instantiation, so the graph form carries none of its end protocol (with it inline the
// pipelined step measured 2.82 vs 2.38 us, same box: profiles/r04w_stream_serve_split_ab.txt)
template <typename WT, int KS, bool SERVE>
__global__ __launch_bounds__(kThreads, 1) void stream_pipe_kernel(StreamPipeParams p) {
    constexpr int CWK = kPipeCwK, CWP = kPipeCwP;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ int abort_flag, end_flag;
    __shared__ int rollback_flag;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wg = blockIdx.x;
    const int C = p.C, nb = p.nb, nl = p.nl, Q = p.queue;
    // serve form: downstream waits also watch the end word and may last the expand role's
    // idle budget (frames arrive at the host's pace)
    const unsigned* const endw = SERVE ? p.end_frame : nullptr;
    const unsigned long long limit = SERVE ? p.fault.spin_ticks + p.idle_ticks : p.fault.spin_ticks;
    const int nE = 2 * nb + 1;
    // per-role parameters selected with compile-time indices (a runtime index into the
    // by-value kernel argument would copy it to scratch)
    int role = -1, gi = 0, gn = 1, N = 0, Kpr = 0, Nout = 0, K0 = 0, d = 1, R = 0, Kps = 0, nparts = 0;
    const void* Wr = nullptr;
    const void* Wsh = nullptr;  // the shrink's weights (the folded last 1x1 reads its columns)
    const float* scr = nullptr;
    const float* shr = nullptr;
#pragma unroll
    for (int l = 0; l < kStreamMaxLayers; ++l) {
        if (l < nl && wg >= p.cu0[l] && wg < p.cu0[l + 1]) {
            role = l;
            gi = wg - p.cu0[l];
            gn = p.cu0[l + 1] - p.cu0[l];
            N = p.N[l];
            Kpr = p.Kp[l];
            Wr = p.W[l];
            scr = p.scale[l];
            shr = p.shift[l];
        }
        if (l == nl - 1) {
            Nout = p.N[l];
            Kps = p.Kp[l];
            Wsh = p.W[l];
        }
        if (l == nl - 2) nparts = p.cu0[l + 1] - p.cu0[l];
    }
    if (role < 0) return;
    // a stream that timed out stays failed until vp3d_stream_reset: no-op launches (no
    // arrival, no position advance), so nothing drifts out of step
    if (__hip_atomic_load(p.fault.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    K0 = p.Kp[0];
    // a role's channels split over its workgroups in units of 8 (one 64-byte line of granules)
    const int nu = (N + 7) >> 3;
    const int c_lo = 8 * (int)((int64_t)nu * gi / gn), c_hi = min(N, 8 * (int)((int64_t)nu * (gi + 1) / gn));
    const int contig = p.row_contig;
    const bool is_expand = role == 0, is_shrink = role == nl - 1;
    const bool is_k = !is_expand && !is_shrink && (role & 1);
    const bool is_p = !is_expand && !is_shrink && !(role & 1);
    // serve form only: the pipelined graph form keeps the shrink role's all-gather (the folded
    // 1x1 stage is its slowest: 2.56 vs 2.46 us/step); serving, the fold takes a layer group
    // and its all-gather off the frame's path (median 24.3 vs 25.2 us)
    const bool fold_p = SERVE && p.fold && role == nl - 2;  // the last block's 1x1: shrink partials out
    const bool fold_s = SERVE && p.fold && is_shrink;       // the shrink role: idle (the host sums)
    const int b = is_k ? (role + 1) / 2 : role / 2;  // block of a k / p role
#pragma unroll
    for (int q = 1; q <= kStreamMaxBlocks; ++q)
        if (q == b && is_k) {
            d = p.dil[q];
            R = p.ring[q];
        }
    if (tid == 0) {
        abort_flag = 0;
        end_flag = 0;
        rollback_flag = 0;
    }

    // ---- LDS carve ----
    float* xbuf = (float*)smem;               // 2 x C: swept input vector, by frame parity
    float* rbuf = xbuf + 2 * C;               // 2 x kPipeMaxCh: residual slice, by parity
    float* scl = rbuf + 2 * kPipeMaxCh;       // kPipeMaxCh scale, then kPipeMaxCh shift
    float* xin = scl + 2 * kPipeMaxCh;        // expand: 2 x kPipeExpandK input vectors, by parity
    float* hist = xin + 2 * kPipeExpandK;     // expand: frames t-1, t-2 (2 x cin0)
    float* ring = hist + 2 * p.cin0;          // k-conv: [wave][R][CWK] partial sums

    float* wring = ring + wid * R * CWK;

    for (int c = c_lo + tid; c < c_hi; c += kThreads) {
        scl[c - c_lo] = scr[c];
        scl[kPipeMaxCh + c - c_lo] = shr[c];
    }
    if (fold_p)  // the folded shrink's channel buffer: slots past c_hi stay zero
        for (int i = tid; i < 64; i += kThreads) xin[i] = 0.f;
    float* gstate = p.state + (int64_t)wg * p.state_stride;
    if (is_k)
        for (int i = tid; i < kWaves * R * CWK; i += kThreads) ring[i] = gstate[i];
    if (is_expand)
        for (int i = tid; i < 2 * p.cin0; i += kThreads) hist[i] = gstate[i];
    const int t0 = *p.frames_seen;
    __syncthreads();

    const int cs = p.chunk_stride;  // granules between 64-granule chunks of an edge
    const int64_t edge_len = (int64_t)(C >> 6) * cs;
    auto edge = [&](int e, int t, int c0 = 0) {
        return EdgeRef{(const gu64*)p.gran + ((int64_t)(t & (Q - 1)) * nE + e) * edge_len, c0, cs};
    };
    auto out_at = [&](int e, int t, int c) {
        return (gu64*)p.gran + ((int64_t)(t & (Q - 1)) * nE + e) * edge_len + (c >> 6) * cs + (c & 63);
    };
    const int pause = p.poll_pause;

    if (is_expand) {
        // ---- lane per channel: row c = c_lo + 64 wid + lane, Kp0 (<= 128) 16-bit weights ----
        const int cin0 = p.cin0;
        const int c = c_lo + wid * 64 + lane;
        f2 w[kPipeExpandK / 2];
#pragma unroll
        for (int i = 0; i < kPipeExpandK / 2; ++i) w[i] = f2{0.f, 0.f};
        if (c < c_hi) {
            const WT* src = (const WT*)Wr + (int64_t)c * K0;
#pragma unroll
            for (int i = 0; i < kPipeExpandK / 2; ++i) w[i] = 2 * i < K0 ? wpair<WT>(src, i) : f2{0.f, 0.f};  // K0 <= kPipeExpandK
        }
        const float sc = c < c_hi ? scl[c - c_lo] : 0.f, sh = c < c_hi ? scl[kPipeMaxCh + c - c_lo] : 0.f;
        // thread i < cin0 owns input element i: frames t-1, t-2 of it stay in registers (hist
        // in LDS only carries them across launches); the padding of both input buffers is
        // written once
        float hp1 = tid < cin0 ? hist[tid] : 0.f, hp2 = tid < cin0 ? hist[cin0 + tid] : 0.f;
        float ph1 = hp1, ph2 = hp2;  // serve: the history before the last frame taken
        unsigned claim_old = 0;      // serve, thread 0: what the commit of the last frame returned
        for (int i = 3 * cin0 + tid; i < 2 * kPipeExpandK; i += kThreads)
            if (i % kPipeExpandK >= 3 * cin0) xin[i] = 0.f;
        for (int s = 0;; ++s) {
            const int t = t0 + s;
            float fv = 0.f;  // element tid (< cin0) of frame t
            if (!SERVE) {
                if (s >= p.steps) break;
                if (tid < cin0) fv = p.frames[(int64_t)(t & (Q - 1)) * cin0 + tid];
            } else {
                // frame t - 1 was taken speculatively: its commit returned an end at or before
                // it -> another expand workgroup ended the launch there (roll t - 1 back below;
                // the commit was issued a frame ago, so this read rarely waits)
                if (tid == 0 && s > 0 && (claim_old & kServeEndBit) && (claim_old & ~kServeEndBit) <= (unsigned)t - 1u) {
                    rollback_flag = 1;
                    end_flag = 1;
                }
                // serve: thread i < cin0 polls granule i of frame t in the host ring (one PCIe
                // round trip brings the value with its tag); thread 0 also ends the launch on a
                // stop request or after idle_ticks without the frame -- if it can claim frame t
                // as the end (no expand workgroup committed t)
                if (tid < cin0) {
                    // (the barrier below also publishes end_flag)
                    const gu64* fg = (const gu64*)p.frame_gran + (int64_t)(t & (Q - 1)) * cin0 + tid;
                    unsigned long long start = __builtin_amdgcn_s_memrealtime();
                    for (;;) {
                        const unsigned long long x = __hip_atomic_load(fg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        if ((unsigned)(x >> 32) == (unsigned)t + 1u) {
                            fv = __uint_as_float((unsigned)x);
                            break;
                        }
                        if (__hip_atomic_load(&end_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                        if (tid == 0) {
                            const unsigned long long now = __builtin_amdgcn_s_memrealtime();
                            if (now - start > kEndCheckTicks &&
                                (__hip_atomic_load(p.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ||
                                 now - start > p.idle_ticks)) {
                                // the host writes a frame's granules before a stop request: a
                                // granule still missing now means frame t was not posted in time
                                const unsigned long long y = __hip_atomic_load(fg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                                if ((unsigned)(y >> 32) == (unsigned)t + 1u) {
                                    fv = __uint_as_float((unsigned)y);
                                    break;
                                }
                                unsigned expect = (unsigned)t;
                                if (__hip_atomic_compare_exchange_strong(p.end_claim, &expect, kServeEndBit | (unsigned)t,
                                                                         __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                                         __HIP_MEMORY_SCOPE_AGENT)) {
                                    // frame t is the end: no expand workgroup took it, and none will
                                    __hip_atomic_store(p.end_frame, (unsigned)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                    __hip_atomic_store(p.ended_host, (unsigned)t + 1u, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_SYSTEM);
                                    __hip_atomic_store(&end_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                    break;
                                }
                                if ((expect & kServeEndBit) && (expect & ~kServeEndBit) <= (unsigned)t) {
                                    // another expand workgroup claimed the end at this frame
                                    __hip_atomic_store(&end_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                                    break;
                                }
                                // another expand workgroup committed frame t (the whole frame was
                                // posted): it arrives, keep polling; the next end check after another
                                // idle period
                                start = now;
                            }
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
            }
            // the 3-frame input vector (frames t-2, t-1, t; the stream start repeats frame 0):
            // the next frame writes the other buffer, and a thread reaches the frame after that
            // only past the next barrier, which every wave passes after its reads of this one
            float* xv = xin + (s & 1) * kPipeExpandK;
            float nh1 = hp1, nh2 = hp2;
            if (tid < cin0) {
                const float v = fv;
                const float h1 = t == 0 ? v : hp1;                        // frame t-1
                const float h2 = t <= 1 ? (t == 0 ? v : h1) : hp2;         // frame t-2
                xv[tid] = h2;
                xv[cin0 + tid] = h1;
                xv[2 * cin0 + tid] = v;
                nh2 = h1;
                nh1 = v;
            }
            __syncthreads();
            if (SERVE && end_flag) {
                // frame t was never posted: the history stays; a rolled-back frame t - 1 leaves
                // no trace (history as before it, its output granules untagged)
                if (rollback_flag) {
                    hp1 = ph1;
                    hp2 = ph2;
                    if (c < c_hi) publish(out_at(0, t - 1, c), 0u, 0.f);
                }
                break;
            }
            ph1 = hp1;
            ph2 = hp2;
            hp1 = nh1;
            hp2 = nh2;
            // serve: commit frame t (speculatively: its outputs go out before the answer,
            // checked at the next frame)
            if (SERVE && tid == 0)
                claim_old = __hip_atomic_fetch_max(p.end_claim, (unsigned)t + 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
            trace_mark(p, wg, s, 0, tid);
            if (c < c_hi) {
                // four independent chains (two v_pk_fma_f32 chains; a 128-deep dependent chain
                // is latency-bound)
                f2 a2[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}};
#pragma unroll
                for (int i = 0; i < kPipeExpandK / 2; ++i)
                    a2[i & 1] = __builtin_elementwise_fma(w[i], *(const f2*)(xv + 2 * i), a2[i & 1]);
                const float a = (a2[0].x + a2[0].y) + (a2[1].x + a2[1].y);
                float y = a * sc + sh;
                y = y > 0.f ? y : 0.f;
                publish(out_at(0, t, c), (unsigned)t + 1u, y);
            }
            trace_mark(p, wg, s, 1, tid);
            // the next frame writes the other xin buffer; hist is rewritten only after the
            // next barrier, which every wave passes after its reads of this frame
        }
        if (tid < cin0) {
            gstate[tid] = hp1;
            gstate[cin0 + tid] = hp2;
        }
    } else if (is_k) {
        // ---- block b's k-conv: CWK rows per wave, NT = 3 taps, k-sliced ----
        f2 w[3][CWK][KS / 2];
        load_rows<WT, 3, CWK, KS>(w, (const WT*)Wr, Kpr, C, c_lo, c_hi, wid, lane, 3, contig);
        // after rows_sum lane l holds row jr = l >> 4 of the wave's rows: lanes 16 jr lead
        const int jr = lane >> 4, jq = jr < CWK ? jr : CWK - 1;
        const int cr = row_of<CWK>(c_lo, wid, jr, contig);
        const bool lead = (lane & 15) == 0 && jr < CWK && cr < c_hi;
        const float sc = lead ? scl[cr - c_lo] : 0.f, sh = lead ? scl[kPipeMaxCh + cr - c_lo] : 0.f;
        Pref pf;
        pref_issue(pf, edge(role - 1, t0), C, tid);
        for (int s = 0; SERVE || s < p.steps; ++s) {
            const int t = t0 + s;
            float* xv = xbuf + (s & 1) * C;
            if (!pref_finish(pf, edge(role - 1, t), C, (unsigned)t + 1u, xv, &abort_flag, p.fault, tid, pause,
                             limit, endw, &end_flag) &&
                !end_flag)
                abort_flag = 1;
            __syncthreads();
            if (abort_flag) return;
            if (end_flag) break;
            trace_mark(p, wg, s, 0, tid);
            if (SERVE || s + 1 < p.steps) pref_issue(pf, edge(role - 1, t + 1), C, tid);  // in flight during this frame
            f2 xl[KS / 2];
            load_x<KS>(xl, xv, lane);
            float vp[CWK];
            lane_dots<3, CWK, KS>(w, xl, 2, vp);
            const float vn = rows_sum<CWK>(vp, lane);  // newest tap, row jr
            const int slot = t & (R - 1);
            if (t == 0) {
                // every tap reads x(0); outputs 1..2d start from the taps that still reach
                // before the stream start
                float v0p[CWK], v1p[CWK];
                lane_dots<3, CWK, KS>(w, xl, 0, v0p);
                lane_dots<3, CWK, KS>(w, xl, 1, v1p);
                const float v0 = rows_sum<CWK>(v0p, lane), v1 = rows_sum<CWK>(v1p, lane);
                const float y = ((v0 + v1) + vn) * sc + sh;
                if (lead) publish(out_at(role, t, cr), (unsigned)t + 1u, y > 0.f ? y : 0.f);
                trace_mark(p, wg, s, 1, tid);
                // ring: all slots zero, then outputs tt = 1..2d from the clamped taps
                for (int i = lane; i < R * CWK; i += 64) wring[i] = 0.f;
                if (lead) {
                    for (int tt = 1; tt <= 2 * d; ++tt) {
                        float a = 0.f;
                        if (2 * d >= tt) a += v0;
                        if (d >= tt) a += v1;
                        wring[(tt & (R - 1)) * CWK + jq] = a;
                    }
                }
            } else {
                const float y = (wring[slot * CWK + jq] + vn) * sc + sh;
                if (lead) publish(out_at(role, t, cr), (unsigned)t + 1u, y > 0.f ? y : 0.f);
                trace_mark(p, wg, s, 1, tid);
                // the older taps of x(t) feed outputs t + d (tap 1) and t + 2d (tap 0)
                float v0p[CWK], v1p[CWK];
                lane_dots<3, CWK, KS>(w, xl, 1, v1p);
                lane_dots<3, CWK, KS>(w, xl, 0, v0p);
                const float v1 = rows_sum<CWK>(v1p, lane), v0 = rows_sum<CWK>(v0p, lane);
                if (lead) {
                    wring[slot * CWK + jq] = 0.f;
                    wring[((t + d) & (R - 1)) * CWK + jq] += v1;
                    wring[((t + 2 * d) & (R - 1)) * CWK + jq] += v0;
                }
            }
        }
        __syncthreads();
        for (int i = tid; i < kWaves * R * CWK; i += kThreads) gstate[i] = ring[i];
    } else if (fold_s) {
        // ---- folded shrink, serving: the host adds the last 1x1's partial sums (nothing to do) ----
    } else {
        // ---- block b's 1x1 conv (+ residual x_b(t)) or the shrink: CWP rows per wave ----
        f2 w[1][CWP][KS / 2];
        load_rows<WT, 1, CWP, KS>(w, (const WT*)Wr, Kpr, C, c_lo, c_hi, wid, lane, 1, contig);
        // folded shrink (the last block's 1x1): thread i sums output o = i >> 3 over the 8
        // channels c_lo + 8 (i & 7) + k of this workgroup (shrink weights in registers)
        const int fo = tid >> 3, fpart = tid & 7;
        float wsh[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int c = c_lo + 8 * fpart + k;
            wsh[k] = fold_p && fo < Nout && c < c_hi ? (float)((const WT*)Wsh)[(int64_t)fo * Kps + c] : 0.f;
        }
        float* ybuf = xin;  // (LDS of the expand role: unused here) this frame's channel outputs
        // after rows_sum lane l holds row l >> 3 of the wave's rows: lanes 8 j lead
        const int cr = row_of<CWP>(c_lo, wid, lane >> 3, contig);
        const bool lead = (lane & 7) == 0 && cr < c_hi;
        const float sc = lead ? scl[cr - c_lo] : 0.f, sh = lead ? scl[kPipeMaxCh + cr - c_lo] : 0.f;
        const int nres = is_p ? c_hi - c_lo : 0;
        Pref pf, pr;
        pref_issue(pr, edge(role - 2, t0, c_lo), nres, tid);
        pref_issue(pf, edge(role - 1, t0), C, tid);
        for (int s = 0; SERVE || s < p.steps; ++s) {
            const int t = t0 + s;
            float* xv = xbuf + (s & 1) * C;
            float* rv = rbuf + (s & 1) * kPipeMaxCh;
            bool ok = pref_finish(pr, edge(role - 2, t, c_lo), nres, (unsigned)t + 1u, rv, &abort_flag, p.fault, tid,
                                  pause, limit, endw, &end_flag);
            if (ok)
                ok = pref_finish(pf, edge(role - 1, t), C, (unsigned)t + 1u, xv, &abort_flag, p.fault, tid,
                                 pause, limit, endw, &end_flag);
            if (!ok && !end_flag) abort_flag = 1;
            __syncthreads();
            if (abort_flag) return;
            if (end_flag) break;
            trace_mark(p, wg, s, 0, tid);
            if (SERVE || s + 1 < p.steps) {  // the next frame's loads are in flight during this one
                pref_issue(pr, edge(role - 2, t + 1, c_lo), nres, tid);
                pref_issue(pf, edge(role - 1, t + 1), C, tid);
            }
            f2 xl[KS / 2];
            load_x<KS>(xl, xv, lane);
            float vp[CWP];
            lane_dots<1, CWP, KS>(w, xl, 0, vp);
            float y = rows_sum<CWP>(vp, lane) * sc + sh;
            if (lead) {
                if (is_p) {
                    y = y > 0.f ? y : 0.f;
                    y += rv[cr - c_lo];
                    if (fold_p)
                        ybuf[cr - c_lo] = y;
                    else
                        publish(out_at(role, t, cr), (unsigned)t + 1u, y);
                } else if (SERVE) {
                    // host-mapped pose ring: the granule's tag tells the host it is there
                    const unsigned long long g = ((unsigned long long)((unsigned)t + 1u) << 32) | __float_as_uint(y);
                    __hip_atomic_store(p.pose_gran + (int64_t)(t & (Q - 1)) * Nout + cr, g, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                } else {
                    p.poses[(int64_t)(t & (Q - 1)) * Nout + cr] = y;
                }
            }
            if (fold_p) {
                // the workgroup's shrink partials: 8 channels per thread (FMA chain in k order),
                // then the 8 threads of an output (lanes 8 j .. 8 j + 7) in a fixed DPP tree;
                // outputs past Nout publish zeros (the granule slots of a workgroup are whole)
                __syncthreads();
                float a = 0.f;
#pragma unroll
                for (int k = 0; k < 8; ++k) a = __builtin_fmaf(wsh[k], ybuf[8 * fpart + k], a);
                a += dpp<0xB1>(a);   // xor 1
                a += dpp<0x4E>(a);   // xor 2
                a += dpp<0x141>(a);  // half mirror: the other quad of the 8 lanes
                if (fpart == 0) {
                    const int64_t slot = (int64_t)(t & (Q - 1)) * (nparts * 64) + gi * 64 + fo;
                    const unsigned long long g = ((unsigned long long)((unsigned)t + 1u) << 32) | __float_as_uint(a);
                    __hip_atomic_store(p.pose_gran + slot, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
            trace_mark(p, wg, s, 1, tid);
        }
    }
    // ---- the last workgroup to finish advances the stream position (every workgroup read
    // t0 above, before its arrival) ----
    __syncthreads();
    if (tid == 0) {
        __threadfence();
        const unsigned prev = atomicAdd((unsigned*)p.arrivals, 1u);
        int active = 0;
#pragma unroll
        for (int l = 0; l <= kStreamMaxLayers; ++l)
            if (l == nl) active = p.cu0[l];
        if (prev == (unsigned)active - 1u) {
            *p.arrivals = 0u;
            const int t_end = SERVE ? (int)__hip_atomic_load(p.end_frame, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                      : t0 + p.steps;
            __hip_atomic_store(p.frames_seen, t_end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

int stream_pipe_lds_bytes(int C, int cin0, int max_ring) {
    return (2 * C + 2 * kPipeMaxCh + 2 * kPipeMaxCh + 2 * kPipeExpandK + 2 * cin0 + kWaves * max_ring * kPipeCwK) * 4;
}

hipError_t launch_stream_pipe(const StreamPipeParams& p, Act wtype, int lds_bytes, hipStream_t s) {
    const dim3 grid(p.cu0[p.nl]);
#define VP3D_PIPE(WT, KS)                                                                                  \
    do {                                                                                                   \
        if (p.serve)                                                                                       \
            hipLaunchKernelGGL((stream_pipe_kernel<WT, KS, true>), grid, dim3(kThreads), lds_bytes, s, p);  \
        else                                                                                               \
            hipLaunchKernelGGL((stream_pipe_kernel<WT, KS, false>), grid, dim3(kThreads), lds_bytes, s, p); \
    } while (0)
    const int KS = p.C / 64;
    if (wtype == Act::F16 && KS == 16) VP3D_PIPE(_Float16, 16);
    else if (wtype == Act::F16 && KS == 4) VP3D_PIPE(_Float16, 4);
    else if (wtype == Act::BF16 && KS == 16) VP3D_PIPE(__bf16, 16);
    else if (wtype == Act::BF16 && KS == 4) VP3D_PIPE(__bf16, 4);
    else if (wtype == Act::F32 && KS == 16) VP3D_PIPE(float, 16);
    else if (wtype == Act::F32 && KS == 4) VP3D_PIPE(float, 4);
    else return hipErrorInvalidValue;
#undef VP3D_PIPE
    return hipGetLastError();
}

bool stream_pipe_channels_ok(int C) { return C == 1024 || C == 256; }

}  // namespace vp3d

namespace vp3d {

hipError_t stream_pipe_prepare(Act wtype, int C, int lds_bytes) {
    const void* f[2] = {nullptr, nullptr};
    if (wtype == Act::F16 && C == 1024) {
        f[0] = (const void*)stream_pipe_kernel<_Float16, 16, false>;
        f[1] = (const void*)stream_pipe_kernel<_Float16, 16, true>;
    } else if (wtype == Act::F16 && C == 256) {
        f[0] = (const void*)stream_pipe_kernel<_Float16, 4, false>;
        f[1] = (const void*)stream_pipe_kernel<_Float16, 4, true>;
    } else if (wtype == Act::BF16 && C == 1024) {
        f[0] = (const void*)stream_pipe_kernel<__bf16, 16, false>;
        f[1] = (const void*)stream_pipe_kernel<__bf16, 16, true>;
    } else if (wtype == Act::BF16 && C == 256) {
        f[0] = (const void*)stream_pipe_kernel<__bf16, 4, false>;
        f[1] = (const void*)stream_pipe_kernel<__bf16, 4, true>;
    } else if (wtype == Act::F32 && C == 1024) {
        f[0] = (const void*)stream_pipe_kernel<float, 16, false>;
        f[1] = (const void*)stream_pipe_kernel<float, 16, true>;
    } else if (wtype == Act::F32 && C == 256) {
        f[0] = (const void*)stream_pipe_kernel<float, 4, false>;
        f[1] = (const void*)stream_pipe_kernel<float, 4, true>;
    } else {
        return hipErrorInvalidValue;
    }
    for (const void* g : f) {
        const hipError_t e = hipFuncSetAttribute(g, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace vp3d
