// Host-side state shared by the C-ABI translation units (vp3d_capi.cpp: eval
// forward + streaming; vp3d_train.cpp: the training step).  Not part of the
// public boundary (include/vp3d.h is).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/vp3d.h"
#include "kernels.h"  // vp3d::SplitCtl (the handle stages its control block)

namespace vp3d {
namespace host {

// Record `msg` as the calling thread's last error (vp3d_last_error) and return `code`.
int fail(int code, const std::string& msg);

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess)                                                           \
            return ::vp3d::host::fail(_e == hipErrorOutOfMemory ? VP3D_ERR_OOM : VP3D_ERR_HIP, \
                                      std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

inline uint16_t f32_to_bf16_rne(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (uint16_t)((u >> 16) | 0x40);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

inline uint16_t f32_to_f16_rne(float f) {
    _Float16 h = (_Float16)f;
    uint16_t r;
    std::memcpy(&r, &h, 2);
    return r;
}

inline float bf16_to_f32(uint16_t h) {
    const uint32_t u = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

inline float f16_to_f32(uint16_t h) {
    _Float16 v;
    std::memcpy(&v, &h, 2);
    return (float)v;
}

// Position of element k (of a K-wide f32 row) in its split-fp16 row of 2K halves:
// 32-wide groups stored [hi(32) | lo(32)] (lo at +32).
inline size_t x3_pos(size_t k) { return (k >> 5) * 64 + (k & 31); }

// One convolution of the stack (expand, k-conv / 1x1 of each block, shrink).
struct Layer {
    int cin = 0, cout = 0, taps = 1, dil = 1, stride = 1;  // conv geometry
    int K = 0, Kp = 0, Np = 0, Ktap = 0, gemm_taps = 1;     // GEMM geometry
    bool relu = true;
    bool residual = false;  // 1x1 conv of a block: add the block-input slice
    int res_stride = 1, res_off = 0;
    float* w32 = nullptr;
    uint16_t* wbf = nullptr;
    uint16_t* wh = nullptr;
    float* scale = nullptr;
    float* shift = nullptr;
    // expand conv only (expand_gemm.hip): 16-bit weights with the BN folded in --
    // W * scale rounded once, shift as two 16-bit columns hi + lo at k = K, K + 1 (the
    // kernel's loader feeds them 1.0); null when K + 2 does not fit in Kp
    uint16_t* wfbf = nullptr;
    uint16_t* wfh = nullptr;
    // split-fp16 path (VP3D_DTYPE_F16X3, every layer; the shrink's since round 6): the f32 weights
    // scaled by 2^e (max |W 2^e| in [2^14, 2^15)) and carried as hi + lo f16 halves,
    // [Np][2 Kp] with each 32-wide K group stored [hi(32) | lo(32)]; scale_x3 = scale * 2^-e
    uint16_t* wx3 = nullptr;
    float* scale_x3 = nullptr;
};

struct ProfEvent {
    int layer;
    hipEvent_t a, b;
    double flop;
};

// Shape rules of TemporalModel.py (validation :20-21, geometry :31,85-124,152-186).
int validate_cfg(const vp3d_cfg* c);
// pad / causal_shift and the per-layer conv + GEMM geometry.
void build_geometry(const vp3d_cfg& c, std::vector<int>& pad, std::vector<int>& causal_shift,
                    std::vector<Layer>& layers);
// Temporal length after each layer for T input frames; false if T does not fit.
bool layer_lengths(const vp3d_cfg& c, const std::vector<int>& pad, const std::vector<Layer>& layers, int T,
                   std::vector<int>& len);

}  // namespace host
}  // namespace vp3d

struct vp3d_handle {
    vp3d_cfg cfg{};
    int device = 0;
    std::vector<int> pad, causal_shift;
    std::vector<vp3d::host::Layer> layers;  // expand, (conv_k, conv_1x1) per block, shrink
    // activation workspace: three rotating buffers
    void* ws = nullptr;
    size_t ws_bytes = 0;
    // window-gather scratch of vp3d_forward_windows when the fused expand path does not apply
    float* gather_ws = nullptr;
    size_t gather_bytes = 0;
    // split-K workspace of conv_gemm_a4 (ConvGemmParams::sk_part / sk_flag), allocated on the
    // first forward whose plan splits a layer; flags zeroed then, each owner unit takes its
    // helpers' counts back out (and vp3d_sync_status re-zeroes them after a reported timeout)
    void* sk_ws = nullptr;
    // host-mapped fault word (vp3d::kFault* bits): a split-K owner unit whose helpers did not
    // arrive in time, a non-finite f16x3 output; checked at the next call and by vp3d_sync_status
    unsigned* sk_err_host = nullptr;
    unsigned* sk_err_dev = nullptr;
    // the split-K control block last written to the device (vp3d::SplitCtl: wait bound, fault
    // word, fault injection), written with the workspace and rewritten when the test knobs
    // change; sk_ctl_stage is the host source of that async copy (per handle: no shared static)
    unsigned long long sk_ctl_spin = 0;
    int sk_ctl_drop = -1;
    vp3d::SplitCtl sk_ctl_stage{};
    // profiling
    bool profiling = false;
    uint64_t prof_mask = ~0ull;  // layers timed while profiling (bit i = layer i)
    std::vector<vp3d::host::ProfEvent> pending;
    std::vector<hipEvent_t> free_events;
    std::vector<double> prof_ms;
    std::vector<int64_t> prof_n;
    std::vector<double> prof_flop;
};
