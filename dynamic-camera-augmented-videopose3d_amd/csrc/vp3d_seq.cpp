// C-ABI of the trajectory-conditioned sequence lifters in eval mode (include/vp3d.h,
// "trajectory lifters"): CoupledTransformer
// (reference common/models/CamTransformer.py:95-205) and CoupledLSTM
// (common/models/CamLSTM.py:47-129), on a batch of windows (forward) or on the
// sliding windows of one sequence (sliding_window, CamTransformer.py:72-92 /
// CamLSTM.py:33-44, called at run.py:713).
//
// Every nn.Linear is a GEMM on the f32 conv-GEMM kernel (bias, ReLU / LeakyReLU,
// a folded eval BatchNorm and the encoder's residual adds in its epilogue); the
// LayerNorms, attention and the LSTM recurrence are seq_lifter.hip.  Frames are
// projected once and shared by every window containing them (sliding windows
// overlap in all but one frame).
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

struct Linear {
    float* w = nullptr;  // [Np][Kp] f32, zero padded
    float* scale = nullptr;
    float* shift = nullptr;
    int N = 0, K = 0, Np = 0, Kp = 0, act = 0;  // act: 0 none, 1 ReLU, 2 LeakyReLU
};

int pad_to(int v, int m) { return (v + m - 1) / m * m; }

}  // namespace

struct vp3d_seq_lifter {
    vp3d_seq_cfg cfg{};
    int device = 0;
    std::vector<float*> allocs;
    Linear in_proj;  // transformer: 46 -> d; lstm: 46 -> 4H (b_ih0 + b_hh0)
    std::vector<Linear> qkv, outp, lin1, lin2, head;
    std::vector<float*> norm1_g, norm1_b, norm2_g, norm2_b;
    float* pe = nullptr;
    float* pre_g = nullptr;
    float* pre_b = nullptr;
    // lstm
    std::vector<float*> wih_t, whh_t, bias;
    float* out_scale = nullptr;
    float* out_shift = nullptr;
    // workspace
    float* ws = nullptr;
    size_t ws_floats = 0;
};

namespace {

int up(vp3d_seq_lifter* h, const std::vector<float>& v, float** out) {
    float* d = nullptr;
    HIP_TRY(hipMalloc(&d, std::max<size_t>(v.size(), 1) * sizeof(float)));
    h->allocs.push_back(d);
    HIP_TRY(hipMemcpy(d, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice));
    *out = d;
    return VP3D_OK;
}

int up_raw(vp3d_seq_lifter* h, const float* v, size_t n, float** out) {
    return up(h, std::vector<float>(v, v + n), out);
}

// nn.Linear (weight (N, K), bias (N)) [-> BatchNorm1d eval (g, b, mean, var)] [-> act]
int make_linear(vp3d_seq_lifter* h, const float* W, const float* bias, int N, int K, const float* const* bn,
                int act, Linear& L) {
    L.N = N;
    L.K = K;
    L.Np = pad_to(N, kPadN);
    L.Kp = pad_to(K, kPadK);
    L.act = act;
    std::vector<float> w((size_t)L.Np * L.Kp, 0.f), sc(N, 1.f), sh(N, 0.f);
    for (int n = 0; n < N; ++n)
        for (int k = 0; k < K; ++k) w[(size_t)n * L.Kp + k] = W[(size_t)n * K + k];
    for (int n = 0; n < N; ++n) {
        const float b = bias ? bias[n] : 0.f;
        if (bn) {
            // (acc + b) * s + t with s = gamma / sqrt(var + eps), t = beta - mean * s
            const float s = bn[0][n] * (1.0f / std::sqrt(bn[3][n] + h->cfg.eps));
            sc[n] = s;
            sh[n] = b * s + (bn[1][n] - bn[2][n] * s);
        } else {
            sh[n] = b;
        }
    }
    int rc = up(h, w, &L.w);
    if (!rc) rc = up(h, sc, &L.scale);
    if (!rc) rc = up(h, sh, &L.shift);
    return rc;
}

// Y[m] = act(A[src(m)] . W^T * scale + shift) [+ R[res(m)]]; rows m < M; A rows of lda floats.
// res(m) = (m / r_T) ... expressed with the conv-GEMM's window mapping: T_out rows per "window".
hipError_t run_linear(const Linear& L, const float* A, int M, int lda, float* Y, int ldy, const float* R, int R_T,
                      int R_off, int T_out, hipStream_t s) {
    ConvGemmParams p{};
    p.A = A;
    p.W = L.w;
    p.scale = L.scale;
    p.shift = L.shift;
    p.R = R;
    p.Y = Y;
    p.M = M;
    p.N = L.N;
    p.K = L.K;
    p.Kp = L.Kp;
    p.T_out = T_out;
    p.T_in = T_out;
    p.stride = 1;
    p.dil = 1;
    p.Ktap = L.K;
    p.lda = lda;
    p.R_T = R_T;
    p.R_stride = 1;
    p.R_off = R_off;
    p.ldr = L.N;
    p.ldy = ldy;
    p.relu = L.act;
    return launch_conv_gemm(p, Act::F32, Act::F32, Act::F32, s);
}

hipError_t run_linear(const Linear& L, const float* A, int M, float* Y, hipStream_t s) {
    return run_linear(L, A, M, L.K, Y, L.N, nullptr, 0, 0, M, s);
}

int expected_weights(const vp3d_seq_cfg* c) {
    if (c->kind == VP3D_SEQ_TRANSFORMER) return 2 + 1 + 2 + 12 * c->num_layers + 2 * (c->n_head_layers + 1);
    return 4 * c->num_layers + 4 + 6 * c->n_head_layers + 2;
}

int validate(const vp3d_seq_cfg* c) {
    if (!c) return fail(VP3D_ERR_ARG, "cfg is NULL");
    if (c->kind != VP3D_SEQ_TRANSFORMER && c->kind != VP3D_SEQ_LSTM) return fail(VP3D_ERR_ARG, "unknown kind");
    if (c->num_joints_in <= 0 || c->in_features <= 0 || c->num_joints_out <= 0 || c->out_features <= 0)
        return fail(VP3D_ERR_ASSERT, "joint / feature counts must be positive");
    if (c->n_head_layers < 1 || c->n_head_layers > VP3D_SEQ_MAX_HEAD) return fail(VP3D_ERR_ARG, "1..8 head layers");
    if (c->num_layers < 1) return fail(VP3D_ERR_ARG, "at least one layer / cell");
    if (c->kind == VP3D_SEQ_TRANSFORMER) {
        if (c->d_model % 8 || c->d_model > 1024) return fail(VP3D_ERR_ARG, "d_model: multiple of 8, <= 1024");
        if (c->n_heads < 1 || c->d_model % c->n_heads) return fail(VP3D_ERR_ARG, "d_model % n_heads != 0");
        const int dh = c->d_model / c->n_heads;
        if (dh != 16 && dh != 32 && dh != 64) return fail(VP3D_ERR_ARG, "head dim must be 16, 32 or 64");
        if (c->max_len < 1) return fail(VP3D_ERR_ARG, "max_len (positional-encoding rows) must be positive");
    } else {
        if (c->d_model != 64 && c->d_model != 128) return fail(VP3D_ERR_ARG, "LSTM hidden size must be 64 or 128");
        if (c->num_layers > 4) return fail(VP3D_ERR_ARG, "at most 4 LSTM cells");
    }
    return VP3D_OK;
}

std::vector<float> transpose(const float* W, int N, int K) {  // (N, K) -> (K, N)
    std::vector<float> t((size_t)N * K);
    for (int n = 0; n < N; ++n)
        for (int k = 0; k < K; ++k) t[(size_t)k * N + n] = W[(size_t)n * K + k];
    return t;
}

int build(vp3d_seq_lifter* h, const float* const* w) {
    const vp3d_seq_cfg& c = h->cfg;
    const int cin = c.num_joints_in * c.in_features + 12;
    const int nout = c.num_joints_out * c.out_features;
    const int d = c.d_model;
    int i = 0, rc = 0;
    auto head = [&](bool bn) -> int {
        int k = d;
        for (int j = 0; j < c.n_head_layers; ++j) {
            Linear L;
            const float* W = w[i];
            const float* b = w[i + 1];
            i += 2;
            const float* const* bnp = nullptr;
            if (bn) {
                bnp = w + i;
                i += 4;
            }
            int r = make_linear(h, W, b, c.head_layers[j], k, bnp, 2, L);
            if (r) return r;
            h->head.push_back(L);
            k = c.head_layers[j];
        }
        Linear L;
        int r = make_linear(h, w[i], w[i + 1], nout, k, nullptr, 0, L);
        i += 2;
        if (r) return r;
        h->head.push_back(L);
        return VP3D_OK;
    };
    if (c.kind == VP3D_SEQ_TRANSFORMER) {
        const int ff = c.dim_feedforward;
        if ((rc = make_linear(h, w[0], w[1], d, cin, nullptr, 0, h->in_proj))) return rc;
        if ((rc = up_raw(h, w[2], (size_t)c.max_len * d, &h->pe))) return rc;
        if ((rc = up_raw(h, w[3], d, &h->pre_g)) || (rc = up_raw(h, w[4], d, &h->pre_b))) return rc;
        i = 5;
        for (int l = 0; l < c.num_layers; ++l) {
            Linear q, o, l1, l2;
            if ((rc = make_linear(h, w[i], w[i + 1], 3 * d, d, nullptr, 0, q))) return rc;
            if ((rc = make_linear(h, w[i + 2], w[i + 3], d, d, nullptr, 0, o))) return rc;
            if ((rc = make_linear(h, w[i + 4], w[i + 5], ff, d, nullptr, 1, l1))) return rc;
            if ((rc = make_linear(h, w[i + 6], w[i + 7], d, ff, nullptr, 0, l2))) return rc;
            float *g1, *b1, *g2, *b2;
            if ((rc = up_raw(h, w[i + 8], d, &g1)) || (rc = up_raw(h, w[i + 9], d, &b1)) ||
                (rc = up_raw(h, w[i + 10], d, &g2)) || (rc = up_raw(h, w[i + 11], d, &b2)))
                return rc;
            h->qkv.push_back(q);
            h->outp.push_back(o);
            h->lin1.push_back(l1);
            h->lin2.push_back(l2);
            h->norm1_g.push_back(g1);
            h->norm1_b.push_back(b1);
            h->norm2_g.push_back(g2);
            h->norm2_b.push_back(b2);
            i += 12;
        }
        return head(false);
    }
    // LSTM: per cell weight_ih (4H, in), weight_hh (4H, H), bias_ih, bias_hh
    const int H = d, G = 4 * H;
    for (int l = 0; l < c.num_layers; ++l) {
        const float* wih = w[i];
        const float* whh = w[i + 1];
        const float* bih = w[i + 2];
        const float* bhh = w[i + 3];
        i += 4;
        std::vector<float> b(G);
        for (int k = 0; k < G; ++k) b[k] = bih[k] + bhh[k];
        if (l == 0) {
            if ((rc = make_linear(h, wih, b.data(), G, cin, nullptr, 0, h->in_proj))) return rc;
            h->wih_t.push_back(nullptr);
            h->bias.push_back(nullptr);
        } else {
            float *wt, *bd;
            if ((rc = up(h, transpose(wih, G, H), &wt)) || (rc = up(h, b, &bd))) return rc;
            h->wih_t.push_back(wt);
            h->bias.push_back(bd);
        }
        float* ht;
        if ((rc = up(h, transpose(whh, G, H), &ht))) return rc;
        h->whh_t.push_back(ht);
    }
    // bn_lstm (eval) folded to an affine of the last hidden state
    std::vector<float> sc(H), sh(H);
    for (int u = 0; u < H; ++u) {
        const float s = w[i][u] * (1.0f / std::sqrt(w[i + 3][u] + c.eps));
        sc[u] = s;
        sh[u] = w[i + 1][u] - w[i + 2][u] * s;
    }
    i += 4;
    if ((rc = up(h, sc, &h->out_scale)) || (rc = up(h, sh, &h->out_shift))) return rc;
    return head(true);
}

int ensure_ws(vp3d_seq_lifter* h, size_t floats) {
    if (floats <= h->ws_floats) return VP3D_OK;
    if (h->ws) HIP_TRY(hipFree(h->ws));
    h->ws = nullptr;
    h->ws_floats = 0;
    HIP_TRY(hipMalloc(&h->ws, floats * sizeof(float)));
    h->ws_floats = floats;
    return VP3D_OK;
}

// frames X (n_frames x cin rows); window w = frames [w*win_stride, w*win_stride + W)
int run(vp3d_seq_lifter* h, const float* x2d, const float* xcam, int64_t n_frames, int n_win, int W, int win_stride,
        float* y, hipStream_t s) {
    const vp3d_seq_cfg& c = h->cfg;
    const int f2 = c.num_joints_in * c.in_features;
    const int cin = f2 + 12;
    const int d = c.d_model;
    const int64_t rows = (int64_t)n_win * W;
    if (rows > (int64_t)1 << 31 || n_frames > (int64_t)1 << 31) return fail(VP3D_ERR_ARG, "too many rows");
    size_t need;
    const int hmax = *std::max_element(c.head_layers, c.head_layers + c.n_head_layers);
    if (c.kind == VP3D_SEQ_TRANSFORMER) {
        if (W > c.max_len) return fail(VP3D_ERR_ASSERT, "window longer than the positional encoding");
        const int ff = c.dim_feedforward;
        need = (size_t)n_frames * cin + (size_t)n_frames * d + (size_t)rows * (3 * d + 3 * d + std::max(ff, d)) +
               (size_t)n_win * 2 * std::max(hmax, d);
    } else {
        need = (size_t)n_frames * cin + (size_t)n_frames * 4 * d + (size_t)n_win * 2 * std::max(hmax, d);
    }
    int rc = ensure_ws(h, need);
    if (rc) return rc;
    float* X = h->ws;
    float* cur = X + (size_t)n_frames * cin;
    HIP_TRY(launch_concat_frames(x2d, f2, xcam, 12, n_frames, X, s));
    const int mx = std::max(hmax, d);
    float* hv;  // (n_win x d) input of the head, = bufs[1]
    float* hx;  // two (n_win x mx) buffers
    if (c.kind == VP3D_SEQ_TRANSFORMER) {
        float* P = cur;
        float* Hb = P + (size_t)n_frames * d;          // rows x d
        float* QKV = Hb + (size_t)rows * d;            // rows x 3d
        float* O = QKV + (size_t)rows * 3 * d;         // rows x d
        float* T1 = O + (size_t)rows * d;              // rows x d
        float* F1 = T1 + (size_t)rows * d;             // rows x max(ff, d)
        hx = F1 + (size_t)rows * std::max(c.dim_feedforward, d);
        HIP_TRY(run_linear(h->in_proj, X, (int)n_frames, P, s));
        HIP_TRY(launch_layernorm_rows(P, d, rows, W, win_stride, h->pe, h->pre_g, h->pre_b, c.eps, Hb, s));
        for (int l = 0; l < c.num_layers; ++l) {
            const bool last = l == c.num_layers - 1;
            HIP_TRY(run_linear(h->qkv[l], Hb, (int)rows, QKV, s));
            HIP_TRY(launch_attention(QKV, n_win, W, d, c.n_heads, last ? 1 : 0, O, s));
            const int M = last ? n_win : (int)rows;
            // self-attention out projection + the residual x (row (w, W-1) of Hb for the last layer)
            if (last)
                HIP_TRY(run_linear(h->outp[l], O, M, d, T1, d, Hb, W, W - 1, 1, s));
            else
                HIP_TRY(run_linear(h->outp[l], O, M, d, T1, d, Hb, M, 0, M, s));
            float* H1 = last ? hx : O;  // O is free once projected; hx = head buffer 0
            HIP_TRY(launch_layernorm_rows(T1, d, M, M, 0, nullptr, h->norm1_g[l], h->norm1_b[l], c.eps, H1, s));
            HIP_TRY(run_linear(h->lin1[l], H1, M, F1, s));
            HIP_TRY(run_linear(h->lin2[l], F1, M, c.dim_feedforward, T1, d, H1, M, 0, M, s));
            HIP_TRY(launch_layernorm_rows(T1, d, M, M, 0, nullptr, h->norm2_g[l], h->norm2_b[l], c.eps,
                                          last ? hx + (size_t)n_win * mx : Hb, s));
        }
        hv = hx + (size_t)n_win * mx;
    } else {
        float* Gin = cur;
        hx = Gin + (size_t)n_frames * 4 * d;
        HIP_TRY(run_linear(h->in_proj, X, (int)n_frames, Gin, s));
        LstmParams p{};
        p.gin = Gin;
        p.win_stride = win_stride;
        p.n_win = n_win;
        p.W = W;
        p.H = d;
        p.L = c.num_layers;
        for (int l = 0; l < c.num_layers; ++l) {
            p.wih_t[l] = h->wih_t[l];
            p.whh_t[l] = h->whh_t[l];
            p.bias[l] = h->bias[l];
        }
        p.out_scale = h->out_scale;
        p.out_shift = h->out_shift;
        hv = hx + (size_t)n_win * mx;
        p.out = hv;
        HIP_TRY(launch_lstm(p, s));
    }
    // MLP head: ping-pong between the two (n_win x mx) buffers, the last layer into y
    float* bufs[2] = {hx, hx + (size_t)n_win * mx};
    const float* in = hv;
    for (size_t j = 0; j < h->head.size(); ++j) {
        const bool lastj = j + 1 == h->head.size();
        float* out = lastj ? y : (in == bufs[0] ? bufs[1] : bufs[0]);
        HIP_TRY(run_linear(h->head[j], in, n_win, out, s));
        in = out;
    }
    return VP3D_OK;
}

}  // namespace

extern "C" {

int vp3d_seq_weight_count(const vp3d_seq_cfg* cfg) {
    if (validate(cfg)) return -1;
    return expected_weights(cfg);
}

int vp3d_seq_create(const vp3d_seq_cfg* cfg, const float* const* weights, int n_weights, vp3d_seq_lifter** out) {
    if (!out) return fail(VP3D_ERR_ARG, "out is NULL");
    *out = nullptr;
    int rc = validate(cfg);
    if (rc) return rc;
    if (!weights || n_weights != expected_weights(cfg))
        return fail(VP3D_ERR_ARG, "expected " + std::to_string(expected_weights(cfg)) + " weight arrays");
    for (int i = 0; i < n_weights; ++i)
        if (!weights[i]) return fail(VP3D_ERR_ARG, "weight array " + std::to_string(i) + " is NULL");
    vp3d_seq_lifter* h = new vp3d_seq_lifter();
    h->cfg = *cfg;
    if (h->cfg.eps <= 0.f) h->cfg.eps = 1e-5f;
    hipGetDevice(&h->device);
    rc = build(h, weights);
    if (rc) {
        vp3d_seq_destroy(h);
        return rc;
    }
    *out = h;
    return VP3D_OK;
}

int vp3d_seq_destroy(vp3d_seq_lifter* h) {
    if (!h) return VP3D_OK;
    int prev = 0;
    hipGetDevice(&prev);
    hipSetDevice(h->device);
    for (float* p : h->allocs) hipFree(p);
    hipFree(h->ws);
    hipSetDevice(prev);
    delete h;
    return VP3D_OK;
}

int vp3d_seq_forward(vp3d_seq_lifter* h, const float* x2d, const float* xcam, int B, int T, float* y, void* stream) {
    if (!h || !x2d || !xcam || !y) return fail(VP3D_ERR_ARG, "NULL argument");
    if (B <= 0 || T <= 0) return fail(VP3D_ERR_ASSERT, "batch and frames must be positive");
    int dev = 0;
    hipGetDevice(&dev);
    if (dev != h->device) return fail(VP3D_ERR_STATE, "handle belongs to another device");
    return run(h, x2d, xcam, (int64_t)B * T, B, T, T, y, (hipStream_t)stream);
}

int vp3d_seq_sliding_window(vp3d_seq_lifter* h, const float* x2d, const float* xcam, int L, int window, float* y,
                            void* stream) {
    if (!h || !x2d || !xcam || !y) return fail(VP3D_ERR_ARG, "NULL argument");
    if (window <= 0) return fail(VP3D_ERR_ASSERT, "window must be positive");
    if (L - window + 1 <= 0) return fail(VP3D_ERR_ARG, "window_size larger than sequence length");
    int dev = 0;
    hipGetDevice(&dev);
    if (dev != h->device) return fail(VP3D_ERR_STATE, "handle belongs to another device");
    return run(h, x2d, xcam, L, L - window + 1, window, 1, y, (hipStream_t)stream);
}

}  // extern "C"
