// C-ABI of the training step (include/vp3d.h, "training step"): the train-mode
// forward and the backward of TemporalModel / TemporalModelOptimized1f
// (reference TemporalModel.py:62-76, :126-138, :188-198 in train mode, driven by
// run.py:451-487) and the Adam(amsgrad) update (run.py:662, torch.optim.Adam).
//
// Every convolution is a conv GEMM on the f32 MFMA kernel (conv_gemm.hip) in three
// roles:
//   forward   Z = conv(X)                      packed W [cout][tap*cin + c]
//   dgrad     dX = conv^T(dZ)                  dilated / dense k-convs: a conv over
//             the zero-padded dZ with flipped taps, W' [cin][(taps-1-tap)*cout + o];
//             strided (taps == stride) and 1x1 convs: one GEMM dZ x W'' with
//             W'' [tap*cin + c][cout] whose output rows are exactly dX's rows
//   wgrad     dW = dZ^T x gather(X)            wgrad_f32_kernel (train.hip)
// BatchNorm (batch statistics), ReLU, dropout and the residual add are the
// elementwise / per-channel passes of train.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "host.h"
#include "kernels.h"

using namespace vp3d;
using namespace vp3d::host;

namespace {

constexpr int64_t kWgradPartFloats = 64ll << 20;  // 256 MB of split-K partials at most

int pad_to(int v, int m) { return (v + m - 1) / m * m; }

// dgrad form of a conv layer: 1 = flipped taps over a zero-padded gradient, 2 = one GEMM
int dgrad_mode(const Layer& L) { return (L.taps > 1 && L.stride == 1) ? 1 : 2; }

struct TrainLayer {
    float* wf = nullptr;  // forward pack [Np][Kp]
    float* wd = nullptr;  // dgrad pack [Np_d][Kp_d]
    int Nd = 0, Kd = 0, Np_d = 0, Kp_d = 0;
};

}  // namespace

struct vp3d_trainer {
    vp3d_cfg cfg{};
    int device = 0;
    std::vector<int> pad, causal_shift;
    std::vector<Layer> layers;
    std::vector<TrainLayer> tl;
    float* ones = nullptr;
    float* zeros = nullptr;
    float* bn = nullptr;  // per BN layer: mean, invstd, alpha, shift (C each)
    // (B, T)-sized arena
    char* arena = nullptr;
    size_t arena_bytes = 0;
    int cap_B = 0, cap_T = 0;
    std::vector<float*> Z, Out;  // per conv layer except shrink: pre-BN and post-activation rows
    float* g[3] = {nullptr, nullptr, nullptr};
    float* dZ = nullptr;
    double* red = nullptr;
    float* coef = nullptr;
    float* wpart = nullptr;
    int64_t wpart_floats = 0;  // >= every layer's N * K (one split of weight-gradient partials)
    // latest forward
    bool have_fwd = false;
    int B = 0, T = 0;
    std::vector<int> len;
    const float* x = nullptr;
    float p = 0.f;
    uint64_t seed = 0;
};

namespace {

int check_device(const vp3d_trainer* t) {
    int dev = 0;
    hipGetDevice(&dev);
    if (dev != t->device) return fail(VP3D_ERR_STATE, "trainer belongs to another device");
    return VP3D_OK;
}

float* bn_arr(vp3d_trainer* t, int layer, int which) {
    return t->bn + ((size_t)layer * 4 + which) * t->cfg.channels;
}

// input frames of layer l for an input of T frames
int lin(const vp3d_trainer* t, const std::vector<int>& len, int l, int T) { return l == 0 ? T : len[l - 1]; }

int dz_pad(const Layer& L) { return dgrad_mode(L) == 1 ? (L.taps - 1) * L.dil : 0; }

int reserve(vp3d_trainer* t, int B, int T) {
    std::vector<int> len;
    if (!layer_lengths(t->cfg, t->pad, t->layers, T, len))
        return fail(VP3D_ERR_ARG, "input of " + std::to_string(T) + " frames does not fit the receptive field");
    const int nl = (int)t->layers.size();
    for (int l = 1; l < nl; ++l) {
        const Layer& L = t->layers[l];
        if (dgrad_mode(L) == 2 && L.taps > 1 && lin(t, len, l, T) != L.taps * len[l])
            return fail(VP3D_ERR_ASSERT, "strided training needs input frames = receptive field (T = " +
                                             std::to_string(T) + ")");
    }
    if (t->arena && B <= t->cap_B && T <= t->cap_T) return VP3D_OK;
    const int C = t->cfg.channels;
    size_t floats = 0;
    std::vector<size_t> zoff, ooff;
    int64_t max_rows = 0, max_dz = 0, max_red = 0;
    for (int l = 0; l < nl; ++l) {
        const int64_t M = (int64_t)B * len[l];
        max_rows = std::max<int64_t>(max_rows, M);
        max_rows = std::max<int64_t>(max_rows, (int64_t)B * lin(t, len, l, T));
        if (l < nl - 1) {
            zoff.push_back(floats);
            floats += (size_t)M * C;
            ooff.push_back(floats);
            floats += (size_t)M * C;
            max_dz = std::max<int64_t>(max_dz, (int64_t)B * (len[l] + 2 * dz_pad(t->layers[l])) * C);
        }
        max_red = std::max<int64_t>(max_red, train_reduce_part_doubles(M, std::max(C, t->layers[l].cout)));
    }
    const size_t g_off = floats;
    floats += 3 * (size_t)max_rows * C;
    const size_t dz_off = floats;
    floats += (size_t)max_dz;
    const size_t coef_off = floats;
    floats += 3 * (size_t)C;
    // split-row weight-gradient partials: up to kWgradPartFloats, and never less than one
    // whole N x K partial (the --dense k-conv of a 243-frame, 1024-channel model is
    // 1024 x 163*1024 = 171 M floats; wgrad_splits never goes below one split)
    int64_t max_nk = 0;
    for (int l = 0; l < nl; ++l)
        max_nk = std::max<int64_t>(max_nk, (int64_t)t->layers[l].cout * t->layers[l].taps * t->layers[l].cin);
    const int64_t wpart_floats = std::max<int64_t>(kWgradPartFloats, max_nk);
    const size_t wpart_off = floats;
    floats += (size_t)wpart_floats;
    floats = (floats + 1) & ~(size_t)1;  // 8-byte alignment for the doubles
    const size_t red_off = floats;
    floats += 2 * (size_t)max_red;
    const size_t bytes = floats * sizeof(float);
    if (t->arena) HIP_TRY(hipFree(t->arena));
    t->arena = nullptr;
    t->arena_bytes = 0;
    HIP_TRY(hipMalloc(&t->arena, bytes));
    t->arena_bytes = bytes;
    t->cap_B = B;
    t->cap_T = T;
    float* f = (float*)t->arena;
    t->Z.clear();
    t->Out.clear();
    for (size_t i = 0; i < zoff.size(); ++i) {
        t->Z.push_back(f + zoff[i]);
        t->Out.push_back(f + ooff[i]);
    }
    for (int i = 0; i < 3; ++i) t->g[i] = f + g_off + (size_t)i * max_rows * C;
    t->dZ = f + dz_off;
    t->coef = f + coef_off;
    t->wpart = f + wpart_off;
    t->wpart_floats = wpart_floats;
    t->red = (double*)(f + red_off);
    return VP3D_OK;
}

// param-table index of layer l's conv weight (state_dict order, vp3d_weight_count)
int widx(int l) { return 5 * l; }

ConvGemmParams gemm_base(const vp3d_trainer* t) {
    ConvGemmParams p{};
    p.scale = t->ones;
    p.shift = t->zeros;
    p.relu = 0;
    return p;
}

}  // namespace

extern "C" {

int vp3d_trainer_create(const vp3d_cfg* cfg, vp3d_trainer** out) {
    if (!out) return fail(VP3D_ERR_ARG, "out is NULL");
    *out = nullptr;
    int rc = validate_cfg(cfg);
    if (rc) return rc;
    if (cfg->channels % 4 != 0) return fail(VP3D_ERR_ARG, "channels must be a multiple of 4");
    vp3d_trainer* t = new vp3d_trainer();
    t->cfg = *cfg;
    if (t->cfg.bn_eps <= 0.f) t->cfg.bn_eps = 1e-5f;
    hipGetDevice(&t->device);
    build_geometry(t->cfg, t->pad, t->causal_shift, t->layers);
    const int nl = (int)t->layers.size();
    t->tl.resize(nl);
    int maxN = 0;
    auto cleanup = [&](int code) {
        for (TrainLayer& T : t->tl) {
            hipFree(T.wf);
            hipFree(T.wd);
        }
        hipFree(t->ones);
        hipFree(t->zeros);
        hipFree(t->bn);
        delete t;
        return code;
    };
    for (int l = 0; l < nl; ++l) {
        const Layer& L = t->layers[l];
        TrainLayer& T = t->tl[l];
        if (hipMalloc(&T.wf, (size_t)L.Np * L.Kp * 4) != hipSuccess ||
            hipMemset(T.wf, 0, (size_t)L.Np * L.Kp * 4) != hipSuccess)
            return cleanup(fail(VP3D_ERR_OOM, "weight pack"));
        maxN = std::max(maxN, L.cout);
        if (l == 0) continue;  // the input is data: no dgrad of the expand conv
        if (dgrad_mode(L) == 1) {
            T.Nd = L.cin;
            T.Kd = L.taps * L.cout;
        } else {
            T.Nd = L.taps * L.cin;
            T.Kd = L.cout;
        }
        T.Np_d = pad_to(T.Nd, kPadN);
        T.Kp_d = pad_to(T.Kd, kPadK);
        maxN = std::max(maxN, T.Nd);
        if (hipMalloc(&T.wd, (size_t)T.Np_d * T.Kp_d * 4) != hipSuccess ||
            hipMemset(T.wd, 0, (size_t)T.Np_d * T.Kp_d * 4) != hipSuccess)
            return cleanup(fail(VP3D_ERR_OOM, "dgrad weight pack"));
    }
    std::vector<float> one(maxN, 1.0f);
    if (hipMalloc(&t->ones, maxN * 4) != hipSuccess || hipMalloc(&t->zeros, maxN * 4) != hipSuccess ||
        hipMalloc(&t->bn, (size_t)nl * 4 * t->cfg.channels * 4) != hipSuccess)
        return cleanup(fail(VP3D_ERR_OOM, "trainer constants"));
    hipMemcpy(t->ones, one.data(), maxN * 4, hipMemcpyHostToDevice);
    hipMemset(t->zeros, 0, maxN * 4);
    *out = t;
    return VP3D_OK;
}

int vp3d_trainer_destroy(vp3d_trainer* t) {
    if (!t) return VP3D_OK;
    int prev = 0;
    hipGetDevice(&prev);
    hipSetDevice(t->device);
    for (TrainLayer& T : t->tl) {
        hipFree(T.wf);
        hipFree(T.wd);
    }
    hipFree(t->ones);
    hipFree(t->zeros);
    hipFree(t->bn);
    hipFree(t->arena);
    hipSetDevice(prev);
    delete t;
    return VP3D_OK;
}

int64_t vp3d_train_layer_rows(const vp3d_trainer* t, int layer) {
    if (!t || !t->have_fwd || layer < 0 || layer >= (int)t->len.size()) return -1;
    return (int64_t)t->B * t->len[layer];
}

int vp3d_train_forward(vp3d_trainer* t, float* const* params, int n_params, const float* x, int B, int T,
                       float dropout_p, double momentum, uint64_t seed, float* y, void* stream) {
    if (!t) return fail(VP3D_ERR_ARG, "trainer is NULL");
    if (!params || !x || !y) return fail(VP3D_ERR_ARG, "NULL argument");
    if (B <= 0) return fail(VP3D_ERR_ASSERT, "batch must be positive");
    if (n_params != vp3d_weight_count(&t->cfg))
        return fail(VP3D_ERR_ARG, "expected " + std::to_string(vp3d_weight_count(&t->cfg)) + " parameters");
    for (int i = 0; i < n_params; ++i)
        if (!params[i]) return fail(VP3D_ERR_ARG, "parameter " + std::to_string(i) + " is NULL");
    if (!(dropout_p >= 0.f && dropout_p < 1.f)) return fail(VP3D_ERR_ARG, "dropout p must be in [0, 1)");
    int rc = check_device(t);
    if (rc) return rc;
    rc = reserve(t, B, T);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    const int nl = (int)t->layers.size();
    const int C = t->cfg.channels;
    std::vector<int> len;
    layer_lengths(t->cfg, t->pad, t->layers, T, len);
    t->have_fwd = false;

    for (int l = 0; l < nl; ++l) {
        const Layer& L = t->layers[l];
        HIP_TRY(launch_pack_weights(params[widx(l)], L.cout, L.cin, L.taps, 0, L.Kp, t->tl[l].wf, s));
    }
    for (int l = 0; l < nl; ++l) {
        const Layer& L = t->layers[l];
        const bool last = l == nl - 1;
        ConvGemmParams p = gemm_base(t);
        p.A = l == 0 ? (const void*)x : (const void*)t->Out[l - 1];
        p.W = t->tl[l].wf;
        p.M = B * len[l];
        p.N = L.cout;
        p.K = L.K;
        p.Kp = L.Kp;
        p.T_out = len[l];
        p.T_in = lin(t, len, l, T);
        p.stride = L.stride;
        p.dil = L.dil;
        p.Ktap = L.Ktap;
        p.lda = L.cin;
        p.ldy = L.cout;
        if (last) {
            p.shift = params[widx(l) + 1];  // shrink bias (scale 1, no relu)
            p.Y = y;
        } else {
            p.Y = t->Z[l];
        }
        HIP_TRY(launch_conv_gemm(p, Act::F32, Act::F32, Act::F32, s));
        if (last) break;
        const int64_t M = (int64_t)B * len[l];
        float* const* bp = params + widx(l) + 1;  // weight, bias, running_mean, running_var
        HIP_TRY(launch_bn_train_stats(t->Z[l], M, C, t->red, bp[0], bp[1], t->cfg.bn_eps, momentum, bp[2], bp[3],
                                      bn_arr(t, l, 0), bn_arr(t, l, 1), bn_arr(t, l, 2), bn_arr(t, l, 3), s));
        const float* R = nullptr;
        int R_T = 0;
        if (L.residual) {
            R = t->Out[l - 2];  // block input (TemporalModel.py:132,192)
            R_T = len[l - 2];
        }
        HIP_TRY(launch_bn_act_fwd(t->Z[l], M, C, bn_arr(t, l, 2), bn_arr(t, l, 3), dropout_p, seed, l, R, len[l], R_T,
                                  L.res_stride, L.res_off, t->Out[l], s));
    }
    t->have_fwd = true;
    t->B = B;
    t->T = T;
    t->len = len;
    t->x = x;
    t->p = dropout_p;
    t->seed = seed;
    return VP3D_OK;
}

int vp3d_train_backward(vp3d_trainer* t, float* const* params, int n_params, const float* dy, float* const* grads,
                        void* stream) {
    if (!t) return fail(VP3D_ERR_ARG, "trainer is NULL");
    if (!t->have_fwd) return fail(VP3D_ERR_STATE, "vp3d_train_backward without a forward");
    if (!params || !dy || !grads) return fail(VP3D_ERR_ARG, "NULL argument");
    if (n_params != vp3d_weight_count(&t->cfg)) return fail(VP3D_ERR_ARG, "parameter count mismatch");
    const int nl = (int)t->layers.size();
    for (int l = 0; l < nl; ++l) {
        const bool last = l == nl - 1;
        const int nk = last ? 2 : 3;  // conv weight (+ BN weight, bias) / shrink weight + bias
        for (int j = 0; j < nk; ++j)
            if (!grads[widx(l) + j] || !params[widx(l) + j])
                return fail(VP3D_ERR_ARG, "gradient / parameter " + std::to_string(widx(l) + j) + " is NULL");
    }
    int rc = check_device(t);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    const int C = t->cfg.channels;
    const int B = t->B, T = t->T;
    const std::vector<int>& len = t->len;

    for (int l = 1; l < nl; ++l) {
        const Layer& L = t->layers[l];
        const TrainLayer& TL = t->tl[l];
        HIP_TRY(launch_pack_weights(params[widx(l)], L.cout, L.cin, L.taps, dgrad_mode(L), TL.Kp_d, TL.wd, s));
    }
    auto wgrad = [&](int l, const float* dz, int ldz, int dz_T, int dz_off, float* dW) -> int {
        const Layer& L = t->layers[l];
        WgradParams w{};
        w.dZ = dz;
        w.ldz = ldz;
        w.dz_T = dz_T;
        w.dz_off = dz_off;
        w.X = l == 0 ? t->x : t->Out[l - 1];
        w.cin = L.cin;
        w.T_in = lin(t, len, l, T);
        w.stride = L.stride;
        w.dil = L.dil;
        w.T_out = len[l];
        w.M = (int64_t)B * len[l];
        w.N = L.cout;
        w.K = L.taps * L.cin;
        w.part = t->wpart;
        if ((int64_t)w.N * w.K > t->wpart_floats)
            return fail(VP3D_ERR_STATE, "weight-gradient partial buffer smaller than one N x K split");
        const int S = wgrad_splits(w.M, w.N, w.K, t->wpart_floats);
        HIP_TRY(launch_wgrad(w, S, L.taps, dW, s));
        return VP3D_OK;
    };
    // dgrad of layer l: gradient wrt its input rows (B * lin(l) rows of cin) into `out`
    auto dgrad = [&](int l, const float* dz, int dz_T, float* out) -> int {
        const Layer& L = t->layers[l];
        const TrainLayer& TL = t->tl[l];
        ConvGemmParams p = gemm_base(t);
        p.A = dz;
        p.W = TL.wd;
        p.N = TL.Nd;
        p.K = TL.Kd;
        p.Kp = TL.Kp_d;
        p.lda = L.cout;
        p.ldy = TL.Nd;
        p.Y = out;
        if (dgrad_mode(L) == 1) {
            p.M = B * lin(t, len, l, T);
            p.T_out = lin(t, len, l, T);
            p.T_in = dz_T;
            p.stride = 1;
            p.dil = L.dil;
            p.Ktap = L.dil == 1 ? L.taps * L.cout : L.cout;
        } else {
            p.M = B * len[l];
            p.T_out = len[l];
            p.T_in = len[l];
            p.stride = 1;
            p.dil = 1;
            p.Ktap = L.cout;
        }
        HIP_TRY(launch_conv_gemm(p, Act::F32, Act::F32, Act::F32, s));
        return VP3D_OK;
    };

    // shrink: bias = column sums of dy, weight = dy^T x Out, dOut = dy x W
    const int ls = nl - 1;
    const Layer& SL = t->layers[ls];
    const int64_t Ms = (int64_t)B * len[ls];
    HIP_TRY(launch_colsum(dy, Ms, SL.cout, SL.cout, t->red, grads[widx(ls) + 1], s));
    rc = wgrad(ls, dy, SL.cout, len[ls], 0, grads[widx(ls)]);
    if (rc) return rc;
    int cur = 0;  // g[cur] = gradient wrt Out[l]
    rc = dgrad(ls, dy, len[ls], t->g[cur]);
    if (rc) return rc;
    int block_out = -1;  // buffer holding the gradient of the current block's output
    for (int l = nl - 2; l >= 0; --l) {
        const Layer& L = t->layers[l];
        const int64_t M = (int64_t)B * len[l];
        const int P = l > 0 ? dz_pad(L) : 0;
        const int dz_T = len[l] + 2 * P;
        if (P > 0) HIP_TRY(hipMemsetAsync(t->dZ, 0, (size_t)B * dz_T * C * sizeof(float), s));
        HIP_TRY(launch_bn_train_backward(t->g[cur], t->Z[l], M, C, params[widx(l) + 1], bn_arr(t, l, 2),
                                         bn_arr(t, l, 3), bn_arr(t, l, 0), bn_arr(t, l, 1), t->p, t->seed, l, t->red,
                                         t->coef, grads[widx(l) + 1], grads[widx(l) + 2], len[l], dz_T, P, t->dZ,
                                         s));
        rc = wgrad(l, t->dZ, C, dz_T, P, grads[widx(l)]);
        if (rc) return rc;
        if (l == 0) break;
        int nxt = 0;
        while (nxt == cur || nxt == block_out) ++nxt;
        rc = dgrad(l, t->dZ, dz_T, t->g[nxt]);
        if (rc) return rc;
        if (L.residual) {
            block_out = cur;  // keep dOut of the block until the k-conv's dgrad is done
        } else if (block_out >= 0) {
            // k-conv of a block: its dgrad is the block input's gradient; add the residual path
            const Layer& PW = t->layers[l + 1];
            HIP_TRY(launch_res_grad_add(t->g[nxt], t->g[block_out], (int64_t)B * len[l + 1], C, len[l + 1],
                                        lin(t, len, l, T), PW.res_stride, PW.res_off, s));
            block_out = -1;
        }
        cur = nxt;
    }
    return VP3D_OK;
}

int vp3d_train_dropout_mask(vp3d_trainer* t, int layer, int64_t n_elems, uint8_t* out, void* stream) {
    if (!t || !out) return fail(VP3D_ERR_ARG, "NULL argument");
    if (!t->have_fwd) return fail(VP3D_ERR_STATE, "no forward yet");
    if (layer < 0 || layer >= (int)t->layers.size() - 1) return fail(VP3D_ERR_ARG, "layer out of range");
    HIP_TRY(launch_dropout_mask(t->seed, t->p, layer, n_elems, out, (hipStream_t)stream));
    return VP3D_OK;
}

int vp3d_train_relu_mask(vp3d_trainer* t, int layer, int64_t n_elems, uint8_t* out, void* stream) {
    if (!t || !out) return fail(VP3D_ERR_ARG, "NULL argument");
    if (!t->have_fwd) return fail(VP3D_ERR_STATE, "no forward yet");
    if (layer < 0 || layer >= (int)t->layers.size() - 1) return fail(VP3D_ERR_ARG, "layer out of range");
    const int64_t n = (int64_t)t->B * t->len[layer] * t->cfg.channels;
    if (n_elems != n) return fail(VP3D_ERR_ARG, "n_elems must be rows * channels = " + std::to_string(n));
    HIP_TRY(launch_relu_mask(t->Z[layer], n, t->cfg.channels, bn_arr(t, layer, 2), bn_arr(t, layer, 3), out,
                             (hipStream_t)stream));
    return VP3D_OK;
}

int vp3d_adam_step(int n, float* const* params, const float* const* grads, float* const* exp_avg,
                   float* const* exp_avg_sq, float* const* max_exp_avg_sq, const int64_t* numel, double lr,
                   double beta1, double beta2, double eps, double weight_decay, int64_t step, int amsgrad,
                   void* stream) {
    if (n < 0 || n > kMaxAdamTensors) return fail(VP3D_ERR_ARG, "1..64 tensors per call");
    if (n == 0) return VP3D_OK;
    if (!params || !grads || !exp_avg || !exp_avg_sq || !numel || (amsgrad && !max_exp_avg_sq))
        return fail(VP3D_ERR_ARG, "NULL table");
    if (step < 1) return fail(VP3D_ERR_ARG, "step must be >= 1");
    AdamList L{};
    L.n = n;
    L.block_start[0] = 0;
    for (int i = 0; i < n; ++i) {
        if (!params[i] || !grads[i] || !exp_avg[i] || !exp_avg_sq[i] || (amsgrad && !max_exp_avg_sq[i]))
            return fail(VP3D_ERR_ARG, "NULL tensor " + std::to_string(i));
        L.param[i] = params[i];
        L.grad[i] = grads[i];
        L.exp_avg[i] = exp_avg[i];
        L.exp_avg_sq[i] = exp_avg_sq[i];
        L.max_exp_avg_sq[i] = amsgrad ? max_exp_avg_sq[i] : nullptr;
        L.numel[i] = numel[i];
        L.block_start[i + 1] = L.block_start[i] + (int)((numel[i] + 1023) / 1024);
    }
    // python-float scalars of _single_tensor_adam, rounded to the tensor dtype where ATen does
    const double bc1 = 1.0 - std::pow(beta1, (double)step);
    const double bc2 = 1.0 - std::pow(beta2, (double)step);
    AdamHyper hp{};
    hp.lerp_w = (float)(1.0 - beta1);
    hp.beta2 = (float)beta2;
    hp.one_minus_beta2 = (float)(1.0 - beta2);
    hp.bc2_sqrt = (float)std::sqrt(bc2);
    hp.eps = (float)eps;
    hp.neg_step_size = (float)(-(lr / bc1));
    hp.weight_decay = (float)weight_decay;
    hp.amsgrad = amsgrad ? 1 : 0;
    HIP_TRY(launch_adam(L, hp, (hipStream_t)stream));
    return VP3D_OK;
}

}  // extern "C"
