// Store-pattern microbenchmark (tool, not product): HBM write rate of the output
// patterns the lifter's epilogues can produce, on a (rows x 1024) 16-bit matrix
// of 663,552 rows (the Optimized1f expand output at B = 8192, 1.36 GB).
//   0 contiguous      : 16 B per lane, consecutive lanes consecutive addresses
//   1 chunk128_16B    : workgroup owns 256 rows; per 64-channel chunk each wave
//                       writes 64 rows x 128 B, 8 rows x 128 B per instruction
//   2 chunk128_8B     : same region order, 8 B per lane, 16 rows x 32 B per instr
//   3 chunk128_16B_p  : 16 B per lane, 16 rows x 64 B per instruction
//   4 rowfull_16B     : workgroup owns 64 rows and writes them row-major whole
// Build: hipcc --offload-arch=gfx950 -O3 store_patterns.hip -o store_patterns
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int N = 1024;       // channels (2 KB rows)

__global__ __launch_bounds__(256) void k_contig(u32x4* y, long n16) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n16; i += (long)gridDim.x * 256)
        y[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
}

// one workgroup = 256 rows, 4 waves x 64 rows, 16 chunks of 64 channels
template <typename T>
__device__ __forceinline__ void st(T* p, T v, bool nt) {
    if (nt)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

template <int MODE, bool NT = false>
__global__ __launch_bounds__(256) void k_chunk(char* y, int M) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const long m_wave = (long)blockIdx.x * 256 + wid * 64;
    for (int ch = 0; ch < N / 64; ++ch) {
        const long col = ch * 128;  // bytes
        if (MODE == 1) {
            // 8 lanes per row (8 x 16 B = 128 B), 8 rows per instruction, 8 instructions
            for (int q = 0; q < 8; ++q) {
                const long m = m_wave + q * 8 + (lane >> 3);
                if (m < M) st((u32x4*)(y + m * 2048 + col + (lane & 7) * 16), u32x4{1u, 2u, 3u, (unsigned)ch}, NT);
            }
        } else if (MODE == 2) {
            // MFMA-transposed layout: row l&15, 4 lane groups x 8 B, j = 0..3 blocks of 32 B
            for (int rb = 0; rb < 4; ++rb)
                for (int j = 0; j < 4; ++j) {
                    const long m = m_wave + rb * 16 + (lane & 15);
                    if (m < M) *(u32x2*)(y + m * 2048 + col + j * 32 + (lane >> 4) * 8) = u32x2{1u, (unsigned)ch};
                }
        } else if (MODE == 3) {
            // after permlane16 swaps: row l&15, 64 B per row per instruction
            for (int rb = 0; rb < 4; ++rb)
                for (int jp = 0; jp < 2; ++jp) {
                    const long m = m_wave + rb * 16 + (lane & 15);
                    const int seg = ((lane >> 4) & 1) * 2 + (lane >> 5);  // 0..3 x 16 B
                    if (m < M) st((u32x4*)(y + m * 2048 + col + jp * 64 + seg * 16), u32x4{1u, 2u, 3u, (unsigned)ch}, NT);
                }
        }
        __builtin_amdgcn_s_barrier();
    }
}

// one workgroup = 64 rows written whole (2 KB each), 16 B per lane
__global__ __launch_bounds__(256) void k_rowfull(char* y, int M) {
    const long m0 = (long)blockIdx.x * 64;
    for (int it = 0; it < 64 * 2048 / (256 * 16); ++it) {
        const long off = (long)it * 4096 + threadIdx.x * 16;
        const long m = m0 + off / 2048;
        if (m < M) *(u32x4*)(y + m0 * 2048 + off) = u32x4{1u, 2u, 3u, (unsigned)it};
    }
}

int main(int argc, char** argv) {
    const int M = argc > 1 ? atoi(argv[1]) : 663552;
    const size_t bytes = (size_t)M * N * 2;
    char* y;
    if (hipMalloc(&y, bytes) != hipSuccess) return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[] = {"contiguous", "chunk128_16B", "chunk128_8B", "chunk128_16B_p", "rowfull_16B",
                           "chunk128_16B nt", "chunk128_16B_p nt"};
    for (int mode = 0; mode < 7; ++mode) {
        float best = 1e30f;
        for (int rep = 0; rep < 6; ++rep) {
            hipEventRecord(a, 0);
            switch (mode) {
                case 0: hipLaunchKernelGGL(k_contig, dim3(4096), dim3(256), 0, 0, (u32x4*)y, (long)(bytes / 16)); break;
                case 1: hipLaunchKernelGGL(k_chunk<1>, dim3((M + 255) / 256), dim3(256), 0, 0, y, M); break;
                case 2: hipLaunchKernelGGL(k_chunk<2>, dim3((M + 255) / 256), dim3(256), 0, 0, y, M); break;
                case 3: hipLaunchKernelGGL(k_chunk<3>, dim3((M + 255) / 256), dim3(256), 0, 0, y, M); break;
                case 4: hipLaunchKernelGGL(k_rowfull, dim3((M + 63) / 64), dim3(256), 0, 0, y, M); break;
                case 5: hipLaunchKernelGGL((k_chunk<1, true>), dim3((M + 255) / 256), dim3(256), 0, 0, y, M); break;
                case 6: hipLaunchKernelGGL((k_chunk<3, true>), dim3((M + 255) / 256), dim3(256), 0, 0, y, M); break;
            }
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (rep > 0 && ms < best) best = ms;
        }
        printf("%-16s %8.3f ms  %7.2f TB/s\n", names[mode], best, bytes / (best * 1e-3) / 1e12);
    }
    hipFree(y);
    return 0;
}
