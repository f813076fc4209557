// Internal launch interface between the C-ABI (vp3d_capi.cpp) and the HIP
// kernels.  Not part of the public boundary (include/vp3d.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vp3d {

// One temporal convolution layer of the lifter expressed as a GEMM over rows
// (b, t) of channel-last activations:
//
//   Y[m, n] = epi( sum_{tap, c} X[src(m) + tap*dil, c] * W[n, tap*Ktap + c] )
//   src(m)  = (m / T_out) * T_in + (m % T_out) * stride
//   epi(v)  = [relu](v * scale[n] + shift[n]) [+ R[res(m), n]]
//   res(m)  = (m / T_out) * R_T + (m % T_out) * R_stride + R_off
//
// This covers every convolution in TemporalModel.py:
//   expand_conv (dilated variant)  stride 1,  taps contiguous (one tap of 3*Cin)
//   expand_conv (Optimized1f)      stride w0, taps contiguous
//   layers_conv[2i] (dilated)      stride 1,  3 taps at row offsets {0, d, 2d}
//   layers_conv[2i] (Optimized1f)  stride w,  taps contiguous
//   layers_conv[2i+1] (1x1)        + residual slice (TemporalModel.py:132,192)
//   shrink (1x1 + bias)            scale = 1, shift = bias, no relu
struct ConvGemmParams {
    const void* A;       // activations: f32 or bf16/f16 rows of `lda` elements
    const void* W;       // packed weights [Np][Kp] (f32 or bf16/f16), zero padded
    const float* scale;  // [N]
    const float* shift;  // [N]
    const void* R;       // residual rows (output dtype) or nullptr
    void* Y;             // output rows of `ldy` elements
    int M, N, K, Kp;
    int T_out, T_in, stride, dil, Ktap, lda;
    int R_T, R_stride, R_off, ldr;
    int ldy;
    int relu;  // 0: none, 1: ReLU, 2: LeakyReLU(0.01) (the 16-bit 256x256 kernels: 0/1 only)
    // conv_gemm_a4 only: split-K of a launch's partial last round of 256 x 256 tiles.  The host
    // provides the workspace (sk_part: 256 KiB per helper unit, at most one round of them;
    // sk_flag: one zeroed int per tile of that round); the launcher fills the plan (sk_split 0 =
    // whole tiles only): tiles [0, sk_full) whole, each of the sk_left tiles after them as
    // sk_split units of nk / sk_split K-tiles -- the helper units store their f32 accumulators,
    // the owner unit (the first K range) adds them, in unit order, before its epilogue.
    // expand_gemm reuses sk_full / sk_split for its N split of the partial last round: row
    // blocks [0, sk_full) whole, each later one as sk_split workgroups of a channel range.
    // A tile's flag counts its helpers in and the owner takes S - 1 back out (an atomic
    // subtract, so a helper arriving after a timed-out owner leaves it at 0, not above).  The
    // owner's wait is bounded (SplitCtl::spin_ticks); on the bound it stores 1 into the
    // host-mapped SplitCtl::err (the next call on the handle, or vp3d_sync_status, reports it:
    // the launch's output is wrong, never silently).  The control block sits in the flag area
    // (kSplitCtlOffset), read only on those paths, so the kernel keeps no extra registers.
    float* sk_part;
    int* sk_flag;
    int sk_full, sk_split, sk_left;
};

// split-K control block at byte kSplitCtlOffset of the flag area (ConvGemmParams::sk_flag)
struct SplitCtl {
    unsigned long long spin_ticks;  // the owner's wait bound (100 MHz clock)
    unsigned* err;                  // host-mapped fault word (device view)
    int drop;                       // fault injection (VP3D_A4_SPLIT_DROP=1): helpers skip their count
    int pad;
};

// bytes of the split-K workspace a handle provides (ConvGemmParams::sk_part, then the flags)
constexpr size_t kSplitPartBytes = (size_t)256 * 256 * 1024;  // one round of 256 KiB slots
constexpr size_t kSplitFlagBytes = 4096;
constexpr size_t kSplitCtlOffset = kSplitFlagBytes - 32;  // flags: tiles of one round (<= 256) before it

enum class Act { F32 = 0, BF16 = 1, F16 = 2 };

// A: element type of the activation input; Y/R: element type of the output.
// compute: F32 -> exact f32 MFMA; BF16/F16 -> 16-bit MFMA with f32 accumulate
// (weights in the same 16-bit type).
hipError_t launch_conv_gemm(const ConvGemmParams& p, Act a_type, Act out_type, Act compute,
                            hipStream_t stream);

// 256x256 LDS-DMA family (conv_gemm_big.hip) for the large tap-aligned layers.
bool conv_gemm_big_eligible(const ConvGemmParams& p, Act a_type, Act out_type, Act compute);
hipError_t launch_conv_gemm_big(const ConvGemmParams& p, Act out_type, Act compute,
                                hipStream_t stream);
// Wave-group ping-pong 256x256 kernel with register-direct epilogue (conv_gemm_8p.hip).
bool conv_gemm_8p_eligible(const ConvGemmParams& p, Act a_type, Act out_type, Act compute);
hipError_t launch_conv_gemm_8p(const ConvGemmParams& p, Act compute, hipStream_t stream);
// 64-deep K-tiles staged as whole 128-byte lines, quadrant phases (conv_gemm_q64.hip).
bool conv_gemm_q64_eligible(const ConvGemmParams& p, Act a_type, Act out_type, Act compute);
hipError_t launch_conv_gemm_q64(const ConvGemmParams& p, Act compute, hipStream_t stream);
// One wave per SIMD, 128 x 128 wave tiles, accumulators in named AGPRs (conv_gemm_a4.hip);
// same contract as q64.
bool conv_gemm_a4_eligible(const ConvGemmParams& p, Act a_type, Act out_type, Act compute);
// >= 384 tiles of 256 x 256, or fewer that a split-K plan spreads over every CU
bool conv_gemm_a4_fills(const ConvGemmParams& p);
// true when the launch of this layer on a4 would split its partial last round (the host then
// provides the split-K workspace, sk_part / sk_flag; without it the tiles run whole)
bool conv_gemm_a4_would_split(const ConvGemmParams& p);
constexpr unsigned long long kSplitSpinTicks = 100000000ull;  // 1 s of the 100 MHz clock
hipError_t launch_conv_gemm_a4(const ConvGemmParams& p, Act compute, hipStream_t stream);
// Split-fp16 mode of conv_gemm_a4 (the q64 contract above, N % 256 == 0, >= 384 tiles); the same
// bits as conv_gemm_q64_x3.
bool conv_gemm_a4_x3_eligible(const ConvGemmParams& p, bool out_f32);
hipError_t launch_conv_gemm_a4_x3(const ConvGemmParams& p, bool out_f32, hipStream_t stream);
// Split-K tail of an a4 launch (conv_gemm_tail.hip): rows [m_begin, M) as (N / 64) x S
// K-slices of 256 x 64 over `ncu` CUs, f32 partials in p.sk_part (the split workspace), then
// one reduction launch with a4's epilogue -- the split-fp16 one (x3) or the 16-bit one (bf16 /
// fp16 rows, BN + ReLU [+ residual]).  fits: the shape and (need_ws) the workspace.
bool conv_gemm_tail_fits(const ConvGemmParams& p, int m_begin, int ncu, bool need_ws);
hipError_t launch_conv_gemm_tail_x3(const ConvGemmParams& p, int m_begin, bool out_f32, int ncu,
                                    hipStream_t stream);
hipError_t launch_conv_gemm_tail16(const ConvGemmParams& p, int m_begin, Act compute, int ncu,
                                   hipStream_t stream);
// The f16x3 shrink (N = cout <= 64 poses channels, f32 rows of ldy out, scale / shift without
// ReLU) on the same kernels: every row, 64 columns (W rows past N zero), 2 K-slices, then a
// reduction that writes the N real channels; p.sk_part = the split workspace (rows in chunks
// that fit it)
hipError_t launch_conv_gemm_x3_shrink(const ConvGemmParams& p, hipStream_t stream);
// Split-fp16 mode of conv_gemm_q64 (VP3D_DTYPE_F16X3): A / W / residual rows of f16 halves,
// each 32-wide K group [hi(32) | lo(32)] (Ktap, Kp, lda, ldr in halves); output split
// (ldy halves) or, out_f32, f32 rows (ldy floats).  N % 64 == 0, N <= 1024.
bool conv_gemm_q64_x3_eligible(const ConvGemmParams& p, bool out_f32);
hipError_t launch_conv_gemm_q64_x3(const ConvGemmParams& p, bool out_f32, hipStream_t stream);
// measurement only (VP3D_ABL=7 launches): 10 u64 timestamps/ids per workgroup
hipError_t conv_gemm_8p_set_trace(unsigned long long* buf);
// measurement builds of conv_gemm_a4.hip only (-DVP3D_ABLATION; VP3D_ABL=4 launches)
hipError_t conv_gemm_a4_set_trace(unsigned long long* buf);

// Window source for a forward that gathers its input on the fly (vp3d_forward_windows):
// the B windows are frames [start_b - lead, start_b - lead + window) of device-resident
// sequences, edge-clamped per sequence (ChunkedGenerator, generators.py:92-137), each
// frame = [kps (f2 floats) | cams (12 floats, K.E) if cams != nullptr]
// (CamTransformer.py:187-190).  pairs: (B, 2) int32 (sequence, start).
struct GatherSrc {
    const float* kps = nullptr;
    int f2 = 0;
    const float* cams = nullptr;
    const int64_t* seq_off = nullptr;
    const int32_t* seq_len = nullptr;
    const int32_t* pairs = nullptr;
    int lead = 0;
};

// Expand convolution, 16-bit compute (expand_gemm.hip): reads the f32 input rows
// directly (no packed copy), 256 rows x all channels per workgroup; the gather form
// reads the window frames straight from the sequences.
bool expand_gemm_eligible(const ConvGemmParams& p, Act out_type, Act compute);
hipError_t launch_expand_gemm(const ConvGemmParams& p, Act compute, hipStream_t stream);
bool expand_gather_eligible(const ConvGemmParams& p, const GatherSrc& g, Act out_type, Act compute);
hipError_t launch_expand_gemm_gather(const ConvGemmParams& p, const GatherSrc& g, Act compute,
                                     hipStream_t stream);

// Split-fp16 expand conv (VP3D_DTYPE_F16X3): f32 input rows (or the gather of `g`) split
// into hi / lo halves in registers, Layer::wx3 weights, BN + ReLU in the epilogue, split
// output rows (expand_gemm.hip, X3 mode).
bool expand_gemm_x3_eligible(const ConvGemmParams& p, const GatherSrc* g);
hipError_t launch_expand_gemm_x3(const ConvGemmParams& p, const GatherSrc* g, hipStream_t stream);

// Tile geometry the packer must pad to (rows of W to kPadN, K to kPadK).
constexpr int kPadN = 256;
constexpr int kPadK = 64;

// Causal streaming step (stream_step.hip): one GEMV layer per launch.
struct StreamLayerParams {
    const void* W;            // packed weights [Np][Kp] of the step dtype
    const float* scale;       // [N]
    const float* shift;       // [N]
    int N, K, Kp, cin, taps, dil, relu;
    const float* in;          // input ring (in_R slots of cin floats) or plain vector (in_R == 0)
    int in_R;
    const float* in_frame;    // expand layer: frame queue (in_frame_R slots), slot t read for tap time t
    int in_frame_R;
    float* in_ring_w;         // expand layer: ring slot the new frame is appended to
    const float* res;         // residual ring (block input) or nullptr
    int res_R;
    float* out;               // output ring (out_R slots of N floats) or plain vector
    int out_R;
    int* frames_seen;         // device stream position t
    int advance;              // last layer: the last workgroup to finish does t += 1
    unsigned* done_counter;   // arrival counter for `advance` (zero between steps)
};
hipError_t launch_stream_gemv(const StreamLayerParams& q, Act wtype, hipStream_t s);

// Causal streaming, persistent form (stream_persist.hip): one launch runs `steps` frames;
// workgroup g owns channels [g*CPW, (g+1)*CPW) of every layer with their 16-bit weights
// resident in LDS, the layer outputs handed to every workgroup through {tag, value}
// granules.  Layers: 0 = expand, 2b-1 / 2b = block b's k-conv / 1x1, nl-1 = shrink.
// Bounded-spin fault state of the persistent stream kernels: `err` (device, sticky until
// vp3d_stream_reset) makes every later launch a no-op, `err_host` (host-mapped) lets the
// host refuse further steps without a synchronisation; spin_ticks = the 100 MHz-clock
// budget of one wait (VP3D_STREAM_SPIN_TICKS overrides it: fault-injection tests).
struct StreamFault {
    unsigned* err;
    unsigned* err_host;
    unsigned long long spin_ticks;
};
constexpr unsigned long long kStreamSpinTicks = 25000000ull;  // 0.25 s

constexpr int kStreamMaxLayers = 16;
constexpr int kStreamMaxTaps = 8;
constexpr int kStreamMaxBlocks = 7;
struct StreamPersistParams {
    const void* W[kStreamMaxLayers];       // packed 16-bit weights [Np][Kp], tap-major K
    const float* scale[kStreamMaxLayers];  // folded BatchNorm (shrink: 1 / bias)
    const float* shift[kStreamMaxLayers];
    int Kp[kStreamMaxLayers], N[kStreamMaxLayers];
    int w_off[kStreamMaxLayers];           // LDS byte offset of each layer's CPW weight rows
    int nl, nb, C, CPW, G, cin0;
    int taps[kStreamMaxBlocks + 1], dil[kStreamMaxBlocks + 1], ring[kStreamMaxBlocks + 1];  // per block b >= 1
    int x_off, xin_off, hist_off, part_off, ss_off;  // LDS byte offsets
    int part_floats, state_floats;         // per workgroup
    const float* frames;                   // frame queue (queue slots of cin0 floats)
    int queue;
    float* poses;                          // pose ring (queue slots of N[nl-1] floats)
    int* frames_seen;                      // stream position (read at start, advanced at the end)
    unsigned long long* gran;              // [2nb+1 edges][2 parities][C] granules, zeroed per launch
    StreamFault fault;                     // sticky timeout word (not zeroed per launch)
    float* state;                          // [G][state_floats]: partial-sum rings + frame history
    int steps;
};
int stream_persist_lds_bytes();
hipError_t launch_stream_persist(const StreamPersistParams& p, Act wtype, hipStream_t s);

// Causal streaming, layer-pipelined form (stream_pipe.hip): workgroup g runs ONE layer
// ("role" l = layer index: 0 expand, 2b-1 / 2b block b's k-conv / 1x1, nl-1 shrink) for
// the channels [N_l * i / n_l, N_l * (i+1) / n_l) of its role (i = g - cu0[l], n_l =
// cu0[l+1] - cu0[l]) with their 16-bit weights in VGPRs; layer outputs go to the next
// role's workgroups through {tag = frame + 1, value} granules, slot frame % queue.
constexpr int kPipeCwK = 3;        // k-conv rows per wave (3 taps each)
constexpr int kPipeCwP = 8;        // 1x1 / shrink rows per wave
constexpr int kPipeMaxCh = 512;    // channels per workgroup (expand: one per lane of 8 waves)
constexpr int kPipeExpandK = 128;  // expand K (3 frames x J_in*F, zero-padded)
constexpr int kStreamTraceSlots = 11;  // input complete, one per wave of the 512-thread workgroup, 2 shader clocks
struct StreamPipeParams {
    const void* W[kStreamMaxLayers];       // packed 16-bit weights [Np][Kp], tap-major K
    const float* scale[kStreamMaxLayers];  // folded BatchNorm (shrink: 1 / bias)
    const float* shift[kStreamMaxLayers];
    int Kp[kStreamMaxLayers], N[kStreamMaxLayers];
    int cu0[kStreamMaxLayers + 1];         // role l owns workgroups [cu0[l], cu0[l+1])
    int nl, nb, C, cin0;
    int dil[kStreamMaxBlocks + 1], ring[kStreamMaxBlocks + 1];  // per block b >= 1 (ring: pow2 >= 2d+1)
    const float* frames;                   // frame queue (queue slots of cin0 floats)
    int queue;                             // power of two
    float* poses;                          // pose ring (queue slots of N[nl-1] floats)
    int* frames_seen;                      // stream position (read at start, advanced by the last workgroup)
    unsigned* arrivals;                    // end-of-launch arrival counter (zero between launches)
    unsigned long long* gran;              // [queue][2nb+1 edges][C / 64 chunks x chunk_stride] granules
    int chunk_stride;                      // granules between the 64-granule chunks of an edge (>= 64)
    int poll_pause;                        // s_sleep 1 pauses between polls of a hand-off
    int row_contig;                        // a wave's rows contiguous (1) or kWaves apart (0)
    StreamFault fault;                     // sticky timeout word
    float* state;                          // [workgroups][state_stride]: k-conv rings / expand history
    int state_stride;
    int steps;
    // serve form (vp3d_stream_serve_*): the launch stays resident and takes frames as the
    // host posts them.  Frames and poses travel as 8-byte {tag = frame + 1, f32 value}
    // granules in host-mapped rings (queue slots of cin0 / N[nl-1] granules): the expand role
    // polls the frame granules themselves (no separate count to read first) and the shrink
    // role stores pose granules the host polls (no fence or done word after them).  The
    // expand role ends the launch at the first frame not posted within idle_ticks (100 MHz
    // clock) or once *stop is set, by writing it to *end_frame (device word, all ones while
    // serving); every other role leaves when it reaches that frame.  The expand workgroups
    // agree on that frame through one claim word (*end_claim, = the stream position at
    // serve_begin): each commits a frame it took by an atomic max to frame + 1, an ending
    // workgroup claims frame t by CAS(t -> kServeEndBit | t) -- which fails once any of them
    // committed t -- and a workgroup whose commit returns an end at or before its frame rolls
    // that frame back (output granules untagged, history restored)
    int serve;
    const unsigned long long* frame_gran;
    unsigned long long* pose_gran;
    const unsigned* stop;
    unsigned* end_frame;
    unsigned* end_claim;
    unsigned* ended_host;                  // host-mapped copy of the end frame + 1 (0 while serving)
    unsigned long long idle_ticks;
    // serve form, shrink folded into the last block's 1x1 (fold != 0; round 5): that role's
    // workgroups each sum the shrink over their own channels (Nout partial sums in a fixed
    // order, padded to 64 granules per workgroup) and store them to the host ring pose_gran
    // [queue][n_parts x 64] instead of handing their channels to the shrink role; the host adds
    // the n_parts partials of an output in workgroup order, then the bias.  One layer group
    // and its all-gather fewer on a frame's path (the graph form keeps the shrink role)
    int fold;
    // diagnostics (VP3D_STREAM_TRACE=n at vp3d_stream_create): every workgroup records the
    // 100 MHz clock when the input of its frame s < trace_frames is complete (slot 0) and, per
    // wave w, after the wave's first output store (slot 1 + w):
    // trace[(wg * trace_frames + s) * kStreamTraceSlots + slot]
    unsigned long long* trace;
    int trace_frames;
};
constexpr unsigned kServeEndBit = 0x80000000u;
int stream_pipe_lds_bytes(int C, int cin0, int max_ring);
bool stream_pipe_channels_ok(int C);
hipError_t stream_pipe_prepare(Act wtype, int C, int lds_bytes);  // dynamic-LDS attribute, once
hipError_t launch_stream_pipe(const StreamPipeParams& p, Act wtype, int lds_bytes, hipStream_t s);

// preprocess kernels (preprocess.hip)
hipError_t launch_normalize_screen(const float* x, int64_t n, int w, int h, float* out,
                                   bool inverse, hipStream_t s);
hipError_t launch_normalize_screen_f64(const double* x, int64_t n, double w, double hw, float* out, hipStream_t s);
hipError_t launch_camera_matrices(const float* intr, const int32_t* frame_seq, const double* extr,
                                  int64_t n_frames, float* out, hipStream_t s);
hipError_t launch_world_to_camera(const float* X, int64_t n, const float q[4], const float t[3],
                                  float* out, hipStream_t s);
hipError_t launch_gather_windows(const float* kps, int f2, const float* cams,
                                 const int64_t* seq_off, const int32_t* seq_len,
                                 const int32_t* pairs, int B, int window, int pad, int shift,
                                 float* out, hipStream_t s);
hipError_t launch_pack_rows(const float* x, int M, int T_out, int T_in, int stride, int lda,
                            int K, int Kp, void* out, bool bf16, hipStream_t s);
// The expand conv's GEMM rows in split-fp16 form: row m = (b, t) is the K = taps * cin f32
// values starting at frame t * stride of window b (x: (B, T_in, cin) rows, or gathered from
// the sequences of `g` when x is null), zero padded to Kp and stored as 2 Kp halves
// (32-wide groups [hi | lo]).
hipError_t launch_pack_rows_x3(const float* x, const struct GatherSrc* g, int M, int T_out, int T_in, int stride,
                               int cin, int K, int Kp, void* out, unsigned* fault, hipStream_t s);
hipError_t launch_mpjpe_accumulate(const float* pred, const float* target, int64_t n,
                                   double* acc, hipStream_t s);
hipError_t launch_mpjpe_backward(const float* pred, const float* target, int64_t n, const float* grad_loss,
                                 float* grad_pred, hipStream_t s);
hipError_t launch_project_to_2d(const float* X, int64_t n_cams, int64_t pts_per_cam, const float* params,
                                bool linear, float* out, hipStream_t s);
// metrics.hip: MPJPE / P-MPJPE / N-MPJPE / MPJVE partial sums per (n_frames, J, 3) pair
// non-finite values in y[0, n) -> `bit` ORed into *flag (host-mapped fault word)
hipError_t launch_nonfinite_check(const float* y, int64_t n, unsigned* flag, unsigned bit, hipStream_t s);
// the handle's fault-word bits (vp3d_sync_status)
constexpr unsigned kFaultSplitTimeout = 1u;   // a split-K owner gave up waiting for its helpers
// an f16x3 forward split a value past the f16 range (|x| > 65,504, gemm::x3_range_flag) or
// produced a non-finite pose value
constexpr unsigned kFaultNonFinite = 2u;
hipError_t launch_pose_metrics(const float* pred, const float* target, int64_t n_frames, int J, double* acc,
                               hipStream_t s);

// ---- training step (train.hip, vp3d_train.cpp) ----
// weight gradient of one conv: part[s][n][k] over row splits s (TN GEMM over rows)
struct WgradParams {
    const float* dZ;   // output-gradient rows; row of (b, t) = b*dz_T + t + dz_off, ldz floats each
    int ldz, dz_T, dz_off;
    const float* X;    // layer input rows (cin floats); tap row = b*T_in + t*stride + tap*dil
    int cin, T_in, stride, dil, T_out;
    int64_t M;         // B * T_out
    int N, K;          // cout, taps * cin
    int64_t rows_per_split;
    float* part;       // [S][N][K]
};
constexpr int kMaxAdamTensors = 64;
struct AdamList {
    float* param[kMaxAdamTensors];
    const float* grad[kMaxAdamTensors];
    float* exp_avg[kMaxAdamTensors];
    float* exp_avg_sq[kMaxAdamTensors];
    float* max_exp_avg_sq[kMaxAdamTensors];
    int64_t numel[kMaxAdamTensors];
    int block_start[kMaxAdamTensors + 1];  // 1024 elements per block
    int n;
};
struct AdamHyper {
    float lerp_w, beta2, one_minus_beta2, bc2_sqrt, eps, neg_step_size, weight_decay;
    int amsgrad;
};
int64_t train_reduce_part_doubles(int64_t M, int C);
// mode 0: forward [cout][k*cin+c]; 1: flipped-tap dgrad [cin][(taps-1-k)*cout+o]; 2: [k*cin+c][cout]
hipError_t launch_pack_weights(const float* w, int cout, int cin, int taps, int mode, int Kp, float* out,
                               hipStream_t s);
hipError_t launch_bn_train_stats(const float* Z, int64_t M, int C, double* part, const float* gamma,
                                 const float* beta, float eps, double momentum, float* running_mean,
                                 float* running_var, float* mean, float* invstd, float* alpha, float* shift,
                                 hipStream_t s);
hipError_t launch_bn_act_fwd(const float* Z, int64_t M, int C, const float* alpha, const float* shift, float p,
                             uint64_t seed, int layer, const float* R, int T_out, int R_T, int R_stride, int R_off,
                             float* Y, hipStream_t s);
hipError_t launch_bn_train_backward(const float* dO, const float* Z, int64_t M, int C, const float* gamma,
                                    const float* alpha, const float* shift, const float* mean, const float* invstd,
                                    float p, uint64_t seed, int layer, double* part, float* coef, float* dgamma,
                                    float* dbeta, int T_out, int dz_T, int dz_off, float* dZ, hipStream_t s);
hipError_t launch_colsum(const float* D, int64_t M, int C, int ld, double* part, float* out, hipStream_t s);
hipError_t launch_res_grad_add(float* dIn, const float* dOut, int64_t M, int C, int T_out, int T_in, int rs, int ro,
                               hipStream_t s);
int wgrad_splits(int64_t M, int N, int K, int64_t max_part_floats);
hipError_t launch_wgrad(const WgradParams& p, int S, int taps, float* dW, hipStream_t s);
hipError_t launch_adam(const AdamList& L, const AdamHyper& hp, hipStream_t s);
hipError_t launch_dropout_mask(uint64_t seed, float p, int layer, int64_t n, uint8_t* out, hipStream_t s);
hipError_t launch_relu_mask(const float* Z, int64_t n, int C, const float* alpha, const float* shift, uint8_t* out,
                            hipStream_t s);

// ---- trajectory lifters, eval mode (seq_lifter.hip, vp3d_seq.cpp) ----
struct LstmParams {
    const float* gin;   // layer-0 gate pre-activations per frame: [frame][4H] (x W_ih^T + b_ih + b_hh)
    int win_stride;     // frame of (window w, step t) = w * win_stride + t
    int n_win, W, H, L;
    const float* wih_t[4];  // layer l >= 1: W_ih^T [H][4H]
    const float* whh_t[4];  // W_hh^T [H][4H]
    const float* bias[4];   // layer l >= 1: b_ih + b_hh [4H]
    const float* out_scale; // BatchNorm (eval) of the last hidden state, folded: h * scale + shift
    const float* out_shift;
    float* out;             // [n_win][H]
};
hipError_t launch_concat_frames(const float* a, int fa, const float* b, int fb, int64_t rows, float* out,
                                hipStream_t s);
hipError_t launch_layernorm_rows(const float* X, int d, int64_t n_rows, int W, int win_stride, const float* pe,
                                 const float* gamma, const float* beta, float eps, float* out, hipStream_t s);
hipError_t launch_attention(const float* QKV, int n_win, int W, int d, int heads, int last_only, float* O,
                            hipStream_t s);
hipError_t launch_lstm(const LstmParams& p, hipStream_t s);

}  // namespace vp3d
