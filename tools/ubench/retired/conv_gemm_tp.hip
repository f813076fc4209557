// Persistent 256x256 conv-GEMM with the MFMA issued transposed and a register-
// direct epilogue: the default kernel for the large 1024-channel layers
// (16-bit operands, 16-bit output).
//
// Contract: ConvGemmParams (kernels.h), tap-aligned 16-bit activations; the block
// convolutions and 1x1 convolutions of TemporalModel / TemporalModelOptimized1f
// (reference common/models/TemporalModel.py:113-119, :129-135, :179-181, :191-195).
//
// What it changes against conv_gemm_big.hip (same LDS ring, same swizzle, same
// pinned K-step schedule of 8 groups of 4 v_mfma_f32_16x16x32 with the next step's
// fragment reads and the refill DMA pieces between them):
//   * persistent: grid = min(tiles, CUs), workgroup r walks tiles r, r+G, ... with
//     ONE continuous LDS-DMA stream over (tile, K-step) stages, so the first three
//     K-steps of tile j+1 are in flight while tile j runs its epilogue (the
//     prologue of every tile but the first leaves the critical path);
//   * D = W . A^T: the weight fragment is the MFMA's A operand, so a lane's
//     accumulator holds 4 consecutive OUTPUT CHANNELS of one row (not 4 rows of one
//     channel).  Four v_permlane16_swap per (row block, channel-block pair) give
//     every lane 8 consecutive channels, so BatchNorm affine, ReLU, the residual
//     add and the 16-bit convert run in registers and each lane stores 16 bytes:
//     16 rows x 64 B per store instruction, no LDS staging, no barrier, nothing
//     the next tile's main loop has to wait for except the stores' vmcnt slots;
//   * stores and the residual loads go through a buffer resource: rows past M are
//     dropped by the hardware range check instead of a branch, so every wave issues
//     exactly the same number of vector-memory instructions per tile, which the
//     counted `s_waitcnt vmcnt` after the epilogue relies on;
//   * BatchNorm scale/shift live in LDS (loaded once per workgroup).
#include <cstdlib>
#include <cstring>

#include "gemm_common.h"

namespace vp3d {
namespace {

using namespace gemm;

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int TM = 256, TN = 256, TK = 32;
constexpr int TSLOTS = 4;
constexpr int TSLOT_BYTES = (TM + TN) * TK * 2;  // 32 KiB
constexpr int TRING = TSLOTS * TSLOT_BYTES;      // 128 KiB
constexpr int TPER = 4;                          // DMA pieces per wave per stage (2 A + 2 B)
constexpr int TMAXN = 1024;                      // channels whose scale/shift fit in LDS
constexpr int TEPI_VMEM = 16;                    // stores per wave per tile (8 row blocks x 2)

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <typename CT>
__global__ __launch_bounds__(512, 1) void conv_gemm_tp(ConvGemmParams p) {
    __shared__ __attribute__((aligned(16))) char smem[TRING + 2 * TMAXN * 4];
    float* const s_scale = (float*)(smem + TRING);
    float* const s_shift = s_scale + TMAXN;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wr = wid >> 2, wc = wid & 3;

    for (int i = tid; i < p.N; i += 512) {
        s_scale[i] = p.scale[i];
        s_shift[i] = p.shift[i];
    }

    const int ntn = p.N / TN;
    const int ntiles = ((p.M + TM - 1) / TM) * ntn;
    const int G = gridDim.x;
    const int r = xcd_remap(blockIdx.x, G);
    const int my_tiles = r < ntiles ? (ntiles - r + G - 1) / G : 0;
    const int nk = p.Kp / TK;
    const int S = my_tiles * nk;
    if (S == 0) return;

    const int dma_row = lane >> 2;
    const int dma_c = ((lane & 3) - 2 * ((lane >> 4) & 3)) & 3;
    const CT* A = (const CT*)p.A;
    const CT* W = (const CT*)p.W;

    // ---- issue cursor over (tile, K-step) stages ----
    struct Cursor {
        uint32_t a_row[2];
        int j, k0, tap_off, cin0, b0;
    } cur;
    auto cursor_tile = [&](int j) {
        cur.j = j;
        cur.k0 = 0;
        cur.tap_off = 0;
        cur.cin0 = 0;
        const int t = r + j * G;
        const int tm = t / ntn;
        const int m0 = tm * TM;
        cur.b0 = (t - tm * ntn) * TN * p.Kp;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            int m = m0 + (wid + 8 * q) * 16 + dma_row;
            m = m < p.M ? m : p.M - 1;  // rows past M read a valid row; never stored
            cur.a_row[q] = (uint32_t)src_row(p, m) * (uint32_t)p.lda + dma_c * 8;
        }
    };
    struct StageAddr {
        uint32_t a[2];
        uint32_t b[2];
        int slot;
    };
    auto stage_addr = [&](int g) {
        StageAddr sa;
        const uint32_t ao = cur.tap_off + cur.cin0;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            sa.a[q] = cur.a_row[q] + ao;
            sa.b[q] = (uint32_t)cur.b0 + (uint32_t)(((wid + 8 * q) * 16 + dma_row) * p.Kp) + cur.k0 + dma_c * 8;
        }
        sa.slot = (g % TSLOTS) * TSLOT_BYTES;
        return sa;
    };
    auto cursor_advance = [&]() {
        cur.k0 += TK;
        cur.cin0 += TK;
        if (cur.cin0 == p.Ktap) {
            cur.cin0 = 0;
            cur.tap_off += p.dil * p.lda;
        }
        if (cur.k0 == p.Kp && cur.j + 1 < my_tiles) cursor_tile(cur.j + 1);
    };
    auto dma_piece = [&](const StageAddr& sa, int idx) {
        char* slot = smem + sa.slot;
        if (idx < 2)
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(A + sa.a[idx]),
                                             (lds_ptr_t)(slot + (wid + 8 * idx) * 1024), 16, 0, 0);
        else
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(W + sa.b[idx - 2]),
                                             (lds_ptr_t)(slot + TM * TK * 2 + (wid + 8 * (idx - 2)) * 1024),
                                             16, 0, 0);
    };

    // ---- fragments (same LDS image and swizzle as conv_gemm_big.hip) ----
    const int frag_chunk = ((lane >> 4) + 2 * (((lane & 15) >> 2) & 3)) & 3;
    const int a_frag_off = (wr * 128 + (lane & 15)) * 64 + frag_chunk * 16;
    const int b_frag_off = TM * TK * 2 + (wc * 64 + (lane & 15)) * 64 + frag_chunk * 16;
    struct Frag {
        u32x4 a[8];
        u32x4 b[4];
    };
    auto read_frags = [&](int g, Frag& f) {
        const char* slot = smem + (g % TSLOTS) * TSLOT_BYTES;
#pragma unroll
        for (int j = 0; j < 4; ++j) f.b[j] = *(const u32x4*)(slot + b_frag_off + j * 16 * 64);
#pragma unroll
        for (int i = 0; i < 8; ++i) f.a[i] = *(const u32x4*)(slot + a_frag_off + i * 16 * 64);
    };

    // acc[i][j]: lane holds channels j*16 + 4*(lane>>4) + (0..3) of row i*16 + (lane&15)
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // ---- epilogue: exactly TEPI_VMEM vector-memory instructions per wave (stores)
    // plus, with a residual, 16 loads that are waited for inside ----
    const __amdgpu_buffer_rsrc_t y_rsrc = make_rsrc(p.Y, (uint32_t)((size_t)p.M * p.ldy * sizeof(CT)));
    auto epilogue = [&](int j) {
        const int t = r + j * G;
        const int tm = t / ntn;
        epilogue_tp<CT, 8>(p, acc, tm * TM + wr * 128, (t - tm * ntn) * TN + wc * 64, lane, s_scale, s_shift,
                           y_rsrc);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
    };

    // ---- prologue ----
    cursor_tile(0);
    const int pre = S < TSLOTS - 1 ? S : TSLOTS - 1;
    for (int g = 0; g < pre; ++g) {
        const StageAddr sa = stage_addr(g);
#pragma unroll
        for (int d = 0; d < TPER; ++d) dma_piece(sa, d);
        cursor_advance();
    }
    if (pre >= 3)
        vm_wait<2 * TPER>();
    else if (pre == 2)
        vm_wait<TPER>();
    else
        vm_wait<0>();
    lds_barrier();  // also publishes scale/shift
    Frag f0, f1;
    read_frags(0, f0);

    // ---- one K-step g: wait for stage g+1 (resident before its fragments are read),
    // refill stage g+3, MFMAs of stage g with the reads of g+1 and the refill pieces
    // pinned between the 8 MFMA groups.  `fresh` = steps since the last epilogue:
    // that epilogue's TEPI_VMEM stores are younger than the stages it waits for ----
    int fresh = 3;
    auto step = [&](int g, Frag& cur_f, Frag& nxt) {
        const bool tile_end = (g + 1) % nk == 0;
        const bool prefetch = !tile_end;
        const bool refill = g + TSLOTS - 1 < S;
        if (prefetch) {
            // stages issued so far: min(S, g + 3); younger than g+1: stage g+2 if issued
            if (g + TSLOTS - 2 < S) {
                if (fresh < 2)
                    vm_wait<TPER + TEPI_VMEM>();
                else
                    vm_wait<TPER>();
            } else {
                vm_wait<0>();
            }
            lds_barrier();
        }
        StageAddr sa;
        if (refill) sa = stage_addr(g + TSLOTS - 1);
        const char* nslot = smem + ((g + 1) % TSLOTS) * TSLOT_BYTES;
#pragma unroll
        for (int gi = 0; gi < 8; ++gi) {
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[gi][j] = mfma16<CT>(cur_f.b[j], cur_f.a[gi], acc[gi][j]);
            __builtin_amdgcn_sched_barrier(0);
            if (prefetch) {
                if (gi < 2) {
                    nxt.b[2 * gi] = *(const u32x4*)(nslot + b_frag_off + (2 * gi) * 16 * 64);
                    nxt.b[2 * gi + 1] = *(const u32x4*)(nslot + b_frag_off + (2 * gi + 1) * 16 * 64);
                } else if (gi < 6) {
                    nxt.a[2 * (gi - 2)] = *(const u32x4*)(nslot + a_frag_off + (2 * (gi - 2)) * 16 * 64);
                    nxt.a[2 * (gi - 2) + 1] = *(const u32x4*)(nslot + a_frag_off + (2 * (gi - 2) + 1) * 16 * 64);
                }
            }
            if (refill && gi < TPER) dma_piece(sa, gi);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (refill) cursor_advance();
        ++fresh;
        if (tile_end) {
            epilogue(g / nk);
            fresh = 0;
            if (g + 1 < S) {
                // younger than stage g+1: stages g+2, g+3 (when issued) and the stores
                if (g + 3 < S)
                    vm_wait<2 * TPER + TEPI_VMEM>();
                else if (g + 2 < S)
                    vm_wait<TPER + TEPI_VMEM>();
                else
                    vm_wait<TEPI_VMEM>();
                lds_barrier();
            }
            read_frags(g + 1, nxt);  // past the last stage this reads a stale slot, unused
        }
    };
    for (int g = 0; g < S; g += 2) {
        step(g, f0, f1);
        if (g + 1 < S) step(g + 1, f1, f0);
    }
    vm_wait<0>();
}

}  // namespace

bool conv_gemm_tp_eligible(const ConvGemmParams& p, Act a_type, Act out_type, Act compute) {
    static const bool on = [] {
        const char* e = getenv("VP3D_GEMM");
        return e && strcmp(e, "tp") == 0;
    }();
    if (!on) return false;
    if (compute == Act::F32 || a_type != compute || out_type != compute) return false;
    if (p.Ktap % TK != 0 || p.Kp % TK != 0 || p.lda % 8 != 0) return false;
    if (p.N % TN != 0 || p.N > TMAXN || p.ldy % 8 != 0 || (p.R && p.ldr % 8 != 0)) return false;
    if ((reinterpret_cast<uintptr_t>(p.A) & 15) || (reinterpret_cast<uintptr_t>(p.Y) & 15) ||
        (p.R && (reinterpret_cast<uintptr_t>(p.R) & 15)))
        return false;
    // 32-bit offsets: output bytes (buffer range), A / W element indices
    if ((size_t)p.M * p.ldy * 2 >= (1u << 31)) return false;
    const int64_t tiles = (int64_t)((p.M + TM - 1) / TM) * (p.N / TN);
    return tiles >= 256;
}

hipError_t launch_conv_gemm_tp(const ConvGemmParams& p, Act compute, hipStream_t stream) {
    static int cus = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
            return v;
        return 256;
    }();
    const int tiles = ((p.M + TM - 1) / TM) * (p.N / TN);
    const dim3 grid(tiles < cus ? tiles : cus);
    if (compute == Act::BF16)
        hipLaunchKernelGGL((conv_gemm_tp<__bf16>), grid, dim3(512), 0, stream, p);
    else
        hipLaunchKernelGGL((conv_gemm_tp<_Float16>), grid, dim3(512), 0, stream, p);
    return hipGetLastError();
}

}  // namespace vp3d
