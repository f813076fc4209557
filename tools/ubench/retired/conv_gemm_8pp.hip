// Persistent form of the wave-group ping-pong 256x256 conv-GEMM (conv_gemm_8p.hip):
// one workgroup per CU walks its tiles with ONE continuous LDS-DMA stream, so the
// first K-steps of tile j+1 are in flight while tile j runs its epilogue, and there
// is no per-tile workgroup launch, scale/shift reload or ring prologue.
//
// Contract: ConvGemmParams (kernels.h), tap-aligned 16-bit activations: the block
// convolutions and 1x1 convolutions of TemporalModelOptimized1f / TemporalModel
// (reference common/models/TemporalModel.py:113-119, :129-135, :179-181, :191-195).
//
// Why (tools/ubench/gemm_check 8pt, per-workgroup timestamps of the non-persistent
// kernel, 1x1 layer M = 221,184, K = 1024): per tile 26.3 us in the K loop against
// 2.3 us ring prologue + 4.9 us epilogue-to-retire + 0.85 us launch gap.
//
// Main loop: exactly conv_gemm_8p's (two 16-MFMA phases per K-step, G1 one barrier
// behind G0, counted vmcnt), run over a global stage index x = it * nk + s of all the
// workgroup's tiles: stage x+2's A pieces and stage x+3's B pieces are issued at step x
// whichever tile they belong to.  A tile's epilogue runs right after its last MFMA
// phase; because G1 trails G0 by one barrier, G0's epilogue overlaps G1's last MFMA
// phase and G1's overlaps G0's first phase of the next tile.
//
// vmcnt bookkeeping (per wave; gfx9 retires VMEM ops in issue order, loads and
// stores alike).  At step x (K-step s of its tile) segment B waits for stage x+1,
// whose last op is A(x+1) (issued in segment A of step x-1).  Younger than it:
//   B(x+2) [step x-1], A(x+2) [step x], B(x+3) [step x]           2 + 2 + 2
//   the previous tile's epilogue: 16 stores (+ 16 residual loads) +16 (+16) at s = 0
// minus the pieces that do not exist at the end of the stream.  nk >= 4 throughout.
#include <type_traits>

#include "gemm_common.h"

namespace vp3d {
namespace {

using namespace gemm;

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int PM = 256, PN = 256, PK = 32;
constexpr int PSLOTS = 4;
constexpr int PSLOT_BYTES = (PM + PN) * PK * 2;  // 32 KiB
constexpr int PRING = PSLOTS * PSLOT_BYTES;      // 128 KiB
constexpr int PMAXN = 1024;

__device__ __forceinline__ void barrier_pinned() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

template <int N>
__device__ __forceinline__ void vmw() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// DYN: tiles handed out by per-XCD atomic queues (ctr[0..7]; ctr[8] counts retired
// workgroups, the last one resets the queues for the next launch) instead of the static
// blockIdx.x + it*G walk: a CU that runs fast takes more tiles, as under the hardware
// dispatcher of the non-persistent kernel.  XCD x owns the tiles xcd_remap gives it
// (base_x + k, k < cnt_x); its workgroups start at k = b>>3 and b>>3 + G/8 and then take
// k = 2G/8 + atomicAdd(ctr[x], 1), two tiles ahead (the next tile's A rows and B pieces
// are issued during the current one).
template <typename CT, bool HAS_R, bool DYN = false>
__global__ __launch_bounds__(512, 1) void conv_gemm_8pp(ConvGemmParams p, unsigned* ctr) {
    __shared__ __attribute__((aligned(16))) char smem[PRING + 2 * PMAXN * 4];
    __shared__ int s_fetch;
    float* const s_scale = (float*)(smem + PRING);
    float* const s_shift = s_scale + PMAXN;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wr = wid >> 2, wc = wid & 3;

    for (int i = tid; i < p.N; i += 512) {
        s_scale[i] = p.scale[i];
        s_shift[i] = p.shift[i];
    }

    const int ntn = p.N / PN;
    const int ntm = (p.M + PM - 1) / PM;
    const int ntiles = ntm * ntn;
    const int G = gridDim.x;
    // virtual blocks blockIdx.x + it*G (same XCD as blockIdx.x since G % 8 == 0), each
    // mapped like conv_gemm_8p's blocks
    const int nt = (ntiles - (int)blockIdx.x + G - 1) / G;
    const int nk = p.Kp / PK;
    const int T = nt * nk;  // stages in this workgroup's stream
    auto tile_of = [&](int it, int& m0, int& n0) __attribute__((always_inline)) {
        const int wg = xcd_remap((int)blockIdx.x + it * G, ntiles);
        const int tm = wg / ntn;
        m0 = tm * PM;
        n0 = (wg - tm * ntn) * PN;
    };
    // DYN: tile k of this workgroup's XCD (same tiles xcd_remap assigns to the XCD)
    const int xcd = (int)blockIdx.x & 7;
    const int xq = ntiles >> 3, xr = ntiles & 7;
    const int xbase = (xcd < xr) ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq;
    const int xcnt = (xcd < xr) ? xq + 1 : xq;
    auto tile_k = [&](int k, int& m0, int& n0) __attribute__((always_inline)) {
        const int wg = xbase + k;
        const int tm = wg / ntn;
        m0 = tm * PM;
        n0 = (wg - tm * ntn) * PN;
    };

    const int dma_row = lane >> 2;
    const int dma_c = ((lane & 3) - 2 * ((lane >> 4) & 3)) & 3;
    const CT* A = (const CT*)p.A;
    const CT* W = (const CT*)p.W;
    int b_lane[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) b_lane[q] = ((wid + 8 * q) * 16 + dma_row) * p.Kp + dma_c * 8;

    // A addressing: a_src of the tile whose stages are being issued, a_next of the tile
    // after it (computed at the top of each tile, where the residual is not live; the
    // switch at that tile's stage 0 is then a register copy)
    int a_src[2], a_next[2];
    auto a_rows = [&](int it, int (&dst)[2]) __attribute__((always_inline)) {
        int m0, n0;
        tile_of(it < nt ? it : nt - 1, m0, n0);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            int m = m0 + (wid + 8 * q) * 16 + dma_row;
            m = m < p.M ? m : p.M - 1;  // rows past M read a valid row; never stored
            dst[q] = src_row(p, m);
        }
    };
    auto a_rows_k = [&](int k, int (&dst)[2]) __attribute__((always_inline)) {
        int m0, n0;
        tile_k(k, m0, n0);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            int m = m0 + (wid + 8 * q) * 16 + dma_row;
            m = m < p.M ? m : p.M - 1;
            dst[q] = src_row(p, m);
        }
    };
    const int gx = G >> 3;
    int k_cur = (int)blockIdx.x >> 3;
    int k_nxt = k_cur + gx < xcnt ? k_cur + gx : -1;
    if constexpr (DYN)
        a_rows_k(k_cur, a_src);
    else
        a_rows(0, a_src);
    auto issue_a = [&](int x) __attribute__((always_inline)) {
        const int it = x / nk;
        const int s = x - it * nk;
        if (s == 0 && x > 0) {
            a_src[0] = a_next[0];
            a_src[1] = a_next[1];
        }
        const int k0 = s * PK;
        const int tap = k0 / p.Ktap;
        const int cin = k0 - tap * p.Ktap + dma_c * 8;
        char* slot = smem + (x % PSLOTS) * PSLOT_BYTES;
#pragma unroll
        for (int q = 0; q < 2; ++q)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(A + (int64_t)(a_src[q] + tap * p.dil) * p.lda + cin),
                                             (lds_ptr_t)(slot + (wid + 8 * q) * 1024), 16, 0, 0);
    };
    int it_cur = 0;  // DYN: index of the tile being computed
    auto issue_b = [&](int x) __attribute__((always_inline)) {
        const int it = x / nk;
        const int s = x - it * nk;
        int m0, n0;
        if constexpr (DYN) {
            // stages of the current tile (it == it_cur) or of the next one
            tile_k(it == it_cur ? k_cur : k_nxt, m0, n0);
        } else {
            tile_of(it, m0, n0);
        }
        char* slot = smem + (x % PSLOTS) * PSLOT_BYTES + PM * PK * 2;
        const CT* wb = W + (int64_t)n0 * p.Kp + s * PK;
#pragma unroll
        for (int q = 0; q < 2; ++q)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(wb + b_lane[q]), (lds_ptr_t)(slot + (wid + 8 * q) * 1024),
                                             16, 0, 0);
    };

    const int frag_chunk = ((lane >> 4) + 2 * (((lane & 15) >> 2) & 3)) & 3;
    const int a_frag_off = (wr * 128 + (lane & 15)) * 64 + frag_chunk * 16;
    const int b_frag_off = PM * PK * 2 + (wc * 64 + (lane & 15)) * 64 + frag_chunk * 16;

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // prologue (once per workgroup): stages 0 and 1 whole, the B pieces of stage 2
    issue_a(0);
    issue_b(0);
    issue_a(1);
    issue_b(1);
    issue_b(2);
    vmw<6>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // scale/shift stores
    barrier_pinned();
    if (wr == 1) barrier_pinned();  // G1 runs one barrier interval behind G0

    const __amdgpu_buffer_rsrc_t y_rsrc = make_rsrc(p.Y, (uint32_t)((size_t)p.M * p.ldy * sizeof(CT)));
    constexpr bool has_r = HAS_R;
    u32x4 bf[4], alo[4], ahi[4];

    // One K-step of the stream.  WAIT: the segment-B vmcnt (-1: none, -2: the first step
    // after an epilogue when `after_epi`, else 6).  IA / IB: issue A(x+2) / B(x+3).
    auto step = [&](int x, auto WAIT, bool ia, bool ib, bool after_epi, int m0, int n0)
                    __attribute__((always_inline)) {
        constexpr int wait = decltype(WAIT)::value;
        const char* slot = smem + (x % PSLOTS) * PSLOT_BYTES;
        // ---- segment A: B fragments + A rows 0-63 of stage x; A pieces of stage x+2
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[j] = *(const u32x4*)(slot + b_frag_off + j * 16 * 64);
#pragma unroll
        for (int i = 0; i < 4; ++i) alo[i] = *(const u32x4*)(slot + a_frag_off + i * 16 * 64);
        if (ia) issue_a(x + 2);
        barrier_pinned();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = mfma16<CT>(bf[j], alo[i], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
        barrier_pinned();
        // ---- segment B: A rows 64-127 of stage x; B pieces of stage x+3; wait stage x+1
#pragma unroll
        for (int i = 0; i < 4; ++i) ahi[i] = *(const u32x4*)(slot + a_frag_off + (4 + i) * 16 * 64);
        if (ib) issue_b(x + 3);
        if constexpr (wait == -2) {
            // first K-step after an epilogue: its 16 stores (+ 16 residual loads) are
            // younger than stage x+1's last piece
            if (after_epi && has_r) vmw<38>();
            else if (after_epi) vmw<22>();
            else vmw<6>();
        } else if constexpr (wait >= 0) {
            vmw<wait>();
        }
        barrier_pinned();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[4 + i][j] = mfma16<CT>(bf[j], ahi[i], acc[4 + i][j]);
        __builtin_amdgcn_s_setprio(0);
        barrier_pinned();
    };
    auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    using W_STREAM = std::integral_constant<int, -2>;  // 6, or 22 behind an epilogue's stores
    using W_NONE = std::integral_constant<int, -1>;

    int x = 0;
    if constexpr (DYN) {
        // Tile ids three tiles ahead: the atomic for tile it+3 is issued around tile it's
        // epilogue (before it without a residual: the stores carry no counted wait, so it
        // returns under them; after it with one, whose residual waits would otherwise hold
        // it), published through LDS after K-step 1 of tile it+1 — by then the counted
        // waits have retired it without stalling — and read after that tile's last K-step.
        int k_n2 = k_nxt >= 0 && k_cur + 2 * gx < xcnt ? k_cur + 2 * gx : -1;
        bool pending = false;
        unsigned fetched = 0;
        while (k_nxt >= 0) {
            int m0, n0;
            tile_k(k_cur, m0, n0);
            a_rows_k(k_nxt, a_next);
            step(x, W_STREAM{}, true, true, it_cur > 0, m0, n0);
            ++x;
            for (int s = 1; s < nk; ++s, ++x) {
                step(x, std::integral_constant<int, 6>{}, true, true, false, m0, n0);
                if (s == 1 && pending && tid == 0) {
                    s_fetch = 3 * gx + (int)fetched;
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                }
            }
            if (pending) {
                const int kk = __builtin_amdgcn_readfirstlane(s_fetch);  // wave-uniform: SGPR
                k_n2 = kk < xcnt ? kk : -1;
                pending = false;
            }
            const bool fetch = k_n2 >= 0;  // more tiles may remain on this XCD
            if (!HAS_R && fetch && tid == 0) fetched = atomicAdd(&ctr[xcd], 1u);
            epilogue_tp<CT, 8, false, HAS_R ? 1 : 0>(p, acc, m0 + wr * 128, n0 + wc * 64, lane, s_scale, s_shift,
                                                     y_rsrc);
            if (HAS_R && fetch && tid == 0) fetched = atomicAdd(&ctr[xcd], 1u);
            pending = fetch;
            zero_acc();
            k_cur = k_nxt;
            k_nxt = k_n2;
            k_n2 = -1;  // tile it+3: read during the next tile when pending
            ++it_cur;
        }
        {
            // the last tile: the stream runs out (x + 3 == T at s = nk-3)
            int m0, n0;
            tile_k(k_cur, m0, n0);
            step(x, W_STREAM{}, true, true, it_cur > 0, m0, n0);
            ++x;
            for (int s = 1; s < nk - 3; ++s, ++x) step(x, std::integral_constant<int, 6>{}, true, true, false, m0, n0);
            step(x, std::integral_constant<int, 4>{}, true, false, false, m0, n0);
            step(x + 1, std::integral_constant<int, 0>{}, false, false, false, m0, n0);
            step(x + 2, W_NONE{}, false, false, false, m0, n0);
            epilogue_tp<CT, 8, false, HAS_R ? 1 : 0>(p, acc, m0 + wr * 128, n0 + wc * 64, lane, s_scale, s_shift,
                                                     y_rsrc);
        }
        if (wr == 0) barrier_pinned();  // match G1's extra barrier
        // retire: the last workgroup out resets the queues for the next launch
        if (tid == 0) {
            const unsigned done = atomicAdd(&ctr[8], 1u);
            if (done == (unsigned)G - 1) {
                for (int i = 0; i < 8; ++i) __hip_atomic_store(&ctr[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&ctr[8], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        return;
    }
    // all tiles but the last: every refill exists.  The residual is loaded inside the
    // epilogue (pipelined one 16-row block ahead): held in registers through the last
    // K-steps it would push this kernel past 256 VGPRs.
    for (int it = 0; it + 1 < nt; ++it) {
        int m0, n0;
        tile_of(it, m0, n0);
        a_rows(it + 1, a_next);
        step(x, W_STREAM{}, true, true, it > 0, m0, n0);
        ++x;
        for (int s = 1; s < nk; ++s, ++x) step(x, std::integral_constant<int, 6>{}, true, true, false, m0, n0);
        epilogue_tp<CT, 8, false, HAS_R ? 1 : 0>(p, acc, m0 + wr * 128, n0 + wc * 64, lane, s_scale, s_shift, y_rsrc);
        zero_acc();
    }
    // the last tile: the stream runs out (x + 3 == T at s = nk-3)
    {
        int m0, n0;
        tile_of(nt - 1, m0, n0);
        step(x, W_STREAM{}, true, true, nt > 1, m0, n0);
        ++x;
        for (int s = 1; s < nk - 3; ++s, ++x) step(x, std::integral_constant<int, 6>{}, true, true, false, m0, n0);
        step(x, std::integral_constant<int, 4>{}, true, false, false, m0, n0);  // B(x+2), A(x+2)
        step(x + 1, std::integral_constant<int, 0>{}, false, false, false, m0, n0);
        step(x + 2, W_NONE{}, false, false, false, m0, n0);
        epilogue_tp<CT, 8, false, HAS_R ? 1 : 0>(p, acc, m0 + wr * 128, n0 + wc * 64, lane, s_scale, s_shift, y_rsrc);
    }
    if (wr == 0) barrier_pinned();  // match G1's extra barrier
}

}  // namespace

bool conv_gemm_8pp_eligible(const ConvGemmParams& p, Act a_type, Act out_type, Act compute) {
    if (!conv_gemm_8p_eligible(p, a_type, out_type, compute)) return false;
    return p.Kp / PK >= 4;
}

// per-device tile queues of the DYN variant (9 counters, zeroed once; every launch
// leaves them zeroed)
static unsigned* queue_counters() {
    static unsigned* ctr[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    if (!ctr[dev]) {
        void* q = nullptr;
        if (hipMalloc(&q, 64 * sizeof(unsigned)) != hipSuccess) return nullptr;
        if (hipMemset(q, 0, 64 * sizeof(unsigned)) != hipSuccess) return nullptr;
        ctr[dev] = (unsigned*)q;
    }
    return ctr[dev];
}

hipError_t launch_conv_gemm_8pp(const ConvGemmParams& p, Act compute, hipStream_t stream, bool dyn) {
    static const int cus = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
            return v;
        return 256;
    }();
    const int tiles = ((p.M + PM - 1) / PM) * (p.N / PN);
    // a multiple of 8 (virtual block b + it*G stays on b's XCD); one workgroup per CU
    int g = tiles < cus ? tiles : cus;
    g = g >= 8 ? g & ~7 : g;
    const dim3 grid(g);
    const bool r = p.R != nullptr;
    if (dyn) {
        unsigned* q = queue_counters();
        if (!q) return hipErrorOutOfMemory;
        if (g % 8) return hipErrorInvalidValue;  // XCD queues need G/8 workgroups per XCD
        if (compute == Act::BF16 && r)
            hipLaunchKernelGGL((conv_gemm_8pp<__bf16, true, true>), grid, dim3(512), 0, stream, p, q);
        else if (compute == Act::BF16)
            hipLaunchKernelGGL((conv_gemm_8pp<__bf16, false, true>), grid, dim3(512), 0, stream, p, q);
        else if (r)
            hipLaunchKernelGGL((conv_gemm_8pp<_Float16, true, true>), grid, dim3(512), 0, stream, p, q);
        else
            hipLaunchKernelGGL((conv_gemm_8pp<_Float16, false, true>), grid, dim3(512), 0, stream, p, q);
        return hipGetLastError();
    }
    if (compute == Act::BF16 && r)
        hipLaunchKernelGGL((conv_gemm_8pp<__bf16, true>), grid, dim3(512), 0, stream, p, nullptr);
    else if (compute == Act::BF16)
        hipLaunchKernelGGL((conv_gemm_8pp<__bf16, false>), grid, dim3(512), 0, stream, p, nullptr);
    else if (r)
        hipLaunchKernelGGL((conv_gemm_8pp<_Float16, true>), grid, dim3(512), 0, stream, p, nullptr);
    else
        hipLaunchKernelGGL((conv_gemm_8pp<_Float16, false>), grid, dim3(512), 0, stream, p, nullptr);
    return hipGetLastError();
}

}  // namespace vp3d
