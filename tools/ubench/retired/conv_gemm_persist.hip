// Persistent 256x256 conv-GEMM: one workgroup per CU walks its tiles with ONE
// continuous LDS-DMA stream, so the K-steps of tile j+1 are already in flight
// while tile j runs its epilogue.
//
// Same arithmetic and layout contract as conv_gemm_big.hip (ConvGemmParams,
// tap-aligned 16-bit activations; reference common/models/TemporalModel.py:113-119,
// :179-181) and the same pinned per-K-step schedule (8 groups of 4
// v_mfma_f32_16x16x32 with the next step's fragment reads and the refill DMA
// pieces between them).  What changes is the outer structure:
//   * grid = min(tiles, CUs); workgroup r (XCD-contiguous numbering) owns tiles
//     r, r + G, r + 2G, ... so each round keeps an XCD on 8 M-panels x 4 N-tiles;
//   * the stage counter g runs over (tile, k) pairs of all owned tiles, the ring
//     refill of step g is stage g + 3 whichever tile it belongs to;
//   * the epilogue stages through a dedicated 32 KiB LDS region (the ring keeps
//     its 128 KiB), 16 rows per pass, column-XOR swizzled (conflict-free writes).
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
constexpr int PEPI_ROWS = 16;                    // rows per epilogue pass per wave
constexpr int PEPI_BYTES = 8 * PEPI_ROWS * 64 * 4;  // 32 KiB
constexpr int PPER = 4;                          // DMA pieces per wave per K-step

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <typename CT, typename OT>
__global__ __launch_bounds__(512, 2) void conv_gemm_h16_persist(ConvGemmParams p) {
    __shared__ __attribute__((aligned(16))) char smem[PRING + PEPI_BYTES];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wr = wid >> 2, wc = wid & 3;

    const int ntn = (p.N + PN - 1) / PN;
    const int ntiles = ((p.M + PM - 1) / PM) * ntn;
    const int G = gridDim.x;
    const int r = xcd_remap(blockIdx.x, G);
    const int my_tiles = r < ntiles ? (ntiles - r + G - 1) / G : 0;
    const int nk = p.Kp / PK;
    const int S = my_tiles * nk;
    if (S == 0) return;

    const int dma_row = lane >> 2;
    const int dma_c = ((lane & 3) - 2 * ((lane >> 4) & 3)) & 3;
    const CT* A = (const CT*)p.A;
    const CT* W = (const CT*)p.W;

    // Issue cursor: the next stage to DMA.  Row offsets are recomputed once per
    // tile (the per-lane divisions of src_row), the K position advances by adds.
    // A (< 2^32 elements) and W offsets fit 32-bit element indices.
    struct Cursor {
        uint32_t a_row[2];              // per lane: src_row * lda + 16-byte chunk
        int j, k0, tap_off, cin0, b0;   // tile, K start, tap*dil*lda, channel start, n0*Kp
    } cur_is;
    auto cursor_tile = [&](int j) {
        cur_is.j = j;
        cur_is.k0 = 0;
        cur_is.tap_off = 0;
        cur_is.cin0 = 0;
        const int t = r + j * G;
        const int tm = t / ntn;
        const int m0 = tm * PM;
        cur_is.b0 = (t - tm * ntn) * PN * p.Kp;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            int m = m0 + (wid + 8 * q) * 16 + dma_row;
            m = m < p.M ? m : p.M - 1;
            cur_is.a_row[q] = (uint32_t)src_row(p, m) * (uint32_t)p.lda + dma_c * 8;
        }
    };
    struct StageAddr {
        uint32_t a[2];
        uint32_t b[2];
        int slot;
    };
    // addresses of the cursor's stage (global stage g)
    auto stage_addr = [&](int g) {
        StageAddr sa;
        const uint32_t ao = cur_is.tap_off + cur_is.cin0;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            sa.a[q] = cur_is.a_row[q] + ao;
            sa.b[q] = (uint32_t)cur_is.b0 + (uint32_t)(((wid + 8 * q) * 16 + dma_row) * p.Kp) + cur_is.k0 +
                      dma_c * 8;
        }
        sa.slot = (g % PSLOTS) * PSLOT_BYTES;
        return sa;
    };
    auto cursor_advance = [&]() {
        cur_is.k0 += PK;
        cur_is.cin0 += PK;
        if (cur_is.cin0 == p.Ktap) {
            cur_is.cin0 = 0;
            cur_is.tap_off += p.dil * p.lda;
        }
        if (cur_is.k0 == p.Kp && cur_is.j + 1 < my_tiles) cursor_tile(cur_is.j + 1);
    };
    auto dma_piece = [&](const StageAddr& sa, int idx) {
        char* slot = smem + sa.slot;
        if (idx < 2)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(A + sa.a[idx]),
                                             (lds_ptr_t)(slot + (wid + 8 * idx) * 1024), 16, 0, 0);
        else
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(W + sa.b[idx - 2]),
                                             (lds_ptr_t)(slot + PM * PK * 2 + (wid + 8 * (idx - 2)) * 1024),
                                             16, 0, 0);
    };

    const int frag_chunk = ((lane >> 4) + 2 * (((lane & 15) >> 2) & 3)) & 3;
    const int a_frag_off = (wr * 128 + (lane & 15)) * 64 + frag_chunk * 16;
    const int b_frag_off = PM * PK * 2 + (wc * 64 + (lane & 15)) * 64 + frag_chunk * 16;
    struct Frag {
        u32x4 a[8];
        u32x4 b[4];
    };
    auto read_frags = [&](int g, Frag& f) {
        const char* slot = smem + (g % PSLOTS) * PSLOT_BYTES;
#pragma unroll
        for (int j = 0; j < 4; ++j) f.b[j] = *(const u32x4*)(slot + b_frag_off + j * 16 * 64);
#pragma unroll
        for (int i = 0; i < 8; ++i) f.a[i] = *(const u32x4*)(slot + a_frag_off + i * 16 * 64);
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // ---- epilogue of owned tile j: BN affine, ReLU, residual, 16-byte stores ----
    float* stage = (float*)(smem + PRING) + wid * (PEPI_ROWS * 64);
    auto epilogue = [&](int j) {
        const int t = r + j * G;
        const int tm = t / ntn;
        const int mw = tm * PM + wr * 128;
        const int nw = (t - tm * ntn) * PN + wc * 64;
        const int c8 = lane & 7;
        const int n = nw + c8 * 8;
        const bool nval = n < p.N;
        float sc[8], sh[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            sc[e] = nval ? p.scale[n + e] : 0.f;
            sh[e] = nval ? p.shift[n + e] : 0.f;
        }
#pragma unroll
        for (int pass = 0; pass < 128 / PEPI_ROWS; ++pass) {
#pragma unroll
            for (int ii = 0; ii < PEPI_ROWS / 16; ++ii) {
                const int i = pass * (PEPI_ROWS / 16) + ii;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int row = ii * 16 + (lane >> 4) * 4 + q;
                        const int col = (jj * 16 + (lane & 15)) ^ (((row >> 2) & 1) << 4);
                        stage[row * 64 + col] = acc[i][jj][q];
                    }
            }
            lds_barrier();
#pragma unroll
            for (int q = 0; q < PEPI_ROWS / 8; ++q) {
                const int row = q * 8 + (lane >> 3);
                const int col = (c8 * 8) ^ (((row >> 2) & 1) << 4);
                const f32x4 lo = *(const f32x4*)&stage[row * 64 + col];
                const f32x4 hi = *(const f32x4*)&stage[row * 64 + col + 4];
                const int m = mw + pass * PEPI_ROWS + row;
                if (m < p.M && nval) {
                    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        v[e] = __fadd_rn(__fmul_rn(v[e], sc[e]), sh[e]);
                        if (p.relu) v[e] = v[e] > 0.f ? v[e] : 0.f;
                    }
                    if (p.R) {
                        const int64_t ro = (int64_t)res_row(p, m) * p.ldr + n;
                        if constexpr (sizeof(OT) == 2) {
                            typedef OT ot8 __attribute__((ext_vector_type(8)));
                            const ot8 r8 = __builtin_bit_cast(ot8, *(const u32x4*)((const OT*)p.R + ro));
#pragma unroll
                            for (int e = 0; e < 8; ++e) v[e] += (float)r8[e];
                        } else {
                            const f32x4 r0 = *(const f32x4*)((const float*)p.R + ro);
                            const f32x4 r1 = *(const f32x4*)((const float*)p.R + ro + 4);
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                v[e] += r0[e];
                                v[e + 4] += r1[e];
                            }
                        }
                    }
                    const int64_t yo = (int64_t)m * p.ldy + n;
                    if constexpr (sizeof(OT) == 2) {
                        typedef OT ot8 __attribute__((ext_vector_type(8)));
                        ot8 o;
#pragma unroll
                        for (int e = 0; e < 8; ++e) o[e] = (OT)v[e];
                        *(u32x4*)((OT*)p.Y + yo) = __builtin_bit_cast(u32x4, o);
                    } else {
                        *(f32x4*)((float*)p.Y + yo) = f32x4{v[0], v[1], v[2], v[3]};
                        *(f32x4*)((float*)p.Y + yo + 4) = f32x4{v[4], v[5], v[6], v[7]};
                    }
                }
            }
            lds_barrier();
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
    };

    // ---- prologue ----
    cursor_tile(0);
    const int pre = S < PSLOTS - 1 ? S : PSLOTS - 1;
    for (int g = 0; g < pre; ++g) {
        const StageAddr sa = stage_addr(g);
#pragma unroll
        for (int d = 0; d < PPER; ++d) dma_piece(sa, d);
        cursor_advance();
    }
    if (pre >= 3)
        vm_wait<2 * PPER>();
    else if (pre == 2)
        vm_wait<PPER>();
    else
        vm_wait<0>();
    lds_barrier();
    Frag f0, f1;
    read_frags(0, f0);

    // ---- one K-step: wait for stage g+1, refill stage g+3, MFMAs of g with the
    // reads of g+1 and the refill pieces pinned between the 8 MFMA groups.  The
    // last K-step of a tile runs the epilogue instead of prefetching (the next
    // tile's first fragments are read after it, keeping the epilogue's registers
    // free of a second fragment set) ----
    auto step = [&](int g, Frag& cur, Frag& nxt) {
        // S is a multiple of nk: every step that is not a tile end has a next stage
        const bool tile_end = (g + 1) % nk == 0;
        const bool prefetch = !tile_end;
        const bool refill = g + PSLOTS - 1 < S;
        if (prefetch) {
            // issued so far: min(S, g + 3) stages; after g+1 at most one more in flight
            if (g + PSLOTS - 2 < S)
                vm_wait<PPER>();
            else
                vm_wait<0>();
            lds_barrier();
        }
        StageAddr sa;
        if (refill) sa = stage_addr(g + PSLOTS - 1);
        const char* nslot = smem + ((g + 1) % PSLOTS) * PSLOT_BYTES;
#pragma unroll
        for (int gi = 0; gi < 8; ++gi) {
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[gi][j] = mfma16<CT>(cur.a[gi], cur.b[j], acc[gi][j]);
            __builtin_amdgcn_sched_barrier(0);
            if (prefetch) {
                if (gi < 2) {
                    nxt.b[2 * gi] = *(const u32x4*)(nslot + b_frag_off + (2 * gi) * 16 * 64);
                    nxt.b[2 * gi + 1] = *(const u32x4*)(nslot + b_frag_off + (2 * gi + 1) * 16 * 64);
                } else if (gi < 6) {
                    nxt.a[2 * (gi - 2)] = *(const u32x4*)(nslot + a_frag_off + (2 * (gi - 2)) * 16 * 64);
                    nxt.a[2 * (gi - 2) + 1] =
                        *(const u32x4*)(nslot + a_frag_off + (2 * (gi - 2) + 1) * 16 * 64);
                }
            }
            if (refill && gi < PPER) dma_piece(sa, gi);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (refill) cursor_advance();
        if (tile_end) {
            epilogue(g / nk);
            // stage g+1 landed; the epilogue stores drop out of the count.  nxt is
            // (re)defined on every path so its previous contents are dead here.
            if (g + 1 < S) {
                vm_wait<0>();
                lds_barrier();
            }
            read_frags(g + 1, nxt);
        }
    };
    for (int g = 0; g < S; g += 2) {
        step(g, f0, f1);
        if (g + 1 < S) step(g + 1, f1, f0);
    }
    vm_wait<0>();
}

}  // namespace

hipError_t launch_conv_gemm_persist(const ConvGemmParams& p, Act out_type, Act compute,
                                    hipStream_t stream) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
            cus = v;
    }
    const int tiles = ((p.M + PM - 1) / PM) * ((p.N + PN - 1) / PN);
    const dim3 grid(tiles < cus ? tiles : cus);
    if (compute == Act::BF16) {
        if (out_type == Act::F32)
            hipLaunchKernelGGL((conv_gemm_h16_persist<__bf16, float>), grid, dim3(512), 0, stream, p);
        else
            hipLaunchKernelGGL((conv_gemm_h16_persist<__bf16, __bf16>), grid, dim3(512), 0, stream, p);
    } else {
        if (out_type == Act::F32)
            hipLaunchKernelGGL((conv_gemm_h16_persist<_Float16, float>), grid, dim3(512), 0, stream, p);
        else
            hipLaunchKernelGGL((conv_gemm_h16_persist<_Float16, _Float16>), grid, dim3(512), 0, stream,
                               p);
    }
    return hipGetLastError();
}

}  // namespace vp3d
