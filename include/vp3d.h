/*
 * vp3d.h — C-ABI of the MI355X-native VideoPose3D temporal lifter.
 *
 * This is the drop-in boundary for the reference's hot path
 * (Bart-Weil/Dynamic-Camera-Augmented-VideoPose3D, common/models/TemporalModel.py).
 * The reference is pure Python, so it has no FFI of its own; every entry point
 * below names the Python interface it replaces (file:line in the reference) and
 * is bound from Python with ctypes.
 *
 * Conventions
 *   - Plain pointers and sizes only.  No torch types cross this boundary.
 *   - "device" pointers are HIP device allocations on the handle's device;
 *     "host" pointers are ordinary process memory.
 *   - `stream` is a hipStream_t passed as void* (NULL = the legacy default stream).
 *   - Every function returns VP3D_OK (0) or a VP3D_ERR_* code; the message of the
 *     last failure on the calling thread is available from vp3d_last_error().
 *     The Python shim maps VP3D_ERR_ASSERT to AssertionError (the reference's
 *     `assert` convention, TemporalModel.py:21,63-65) and everything else to
 *     RuntimeError.
 *   - Layouts are channel-last: a (B, T, J, F) pose tensor is already the
 *     (B, T, J*F) activation matrix the first convolution consumes, and the
 *     (B, T', J_out*3) output matrix is already the (B, T', J_out, 3) result.
 */
#ifndef VP3D_H
#define VP3D_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VP3D_ABI_VERSION 1
#define VP3D_MAX_BLOCKS 8

/* status codes */
#define VP3D_OK 0
#define VP3D_ERR_ASSERT 1 /* shape / rank / config violation (reference: assert) */
#define VP3D_ERR_ARG 2    /* bad pointer or argument                          */
#define VP3D_ERR_HIP 3    /* HIP runtime failure                              */
#define VP3D_ERR_OOM 4    /* device allocation failed                         */
#define VP3D_ERR_STATE 5  /* handle misuse (wrong device, not reserved, ...)  */

/* model variants (TemporalModel.py:79 and :141) */
#define VP3D_VARIANT_DILATED 0    /* TemporalModel             */
#define VP3D_VARIANT_STRIDED_1F 1 /* TemporalModelOptimized1f  */

/* arithmetic type of the convolution stack */
#define VP3D_DTYPE_F32 0  /* exact f32 MFMA (v_mfma_f32_16x16x4_f32), the parity path */
#define VP3D_DTYPE_BF16 1 /* bf16 operands, f32 accumulate (v_mfma_f32_16x16x32_bf16) */
#define VP3D_DTYPE_F16 2  /* f16 operands, f32 accumulate (v_mfma_f32_16x16x32_f16)   */
/* split fp16: every f32 operand carried as hi + lo f16 halves (weights pre-scaled by a
 * per-layer power of two), each conv the three products hi.hi + hi.lo + lo.hi on
 * v_mfma_f32_16x16x32_f16 with f32 accumulation -- fp32-level results (the parity gate)
 * at the 16-bit MFMA rate; eval forward only (vp3d_forward / vp3d_forward_windows),
 * channels % 64 == 0 and <= 1024; the shrink runs the exact f32 GEMM */
#define VP3D_DTYPE_F16X3 3

/* Model configuration: the constructor arguments of TemporalModel /
 * TemporalModelOptimized1f (TemporalModel.py:85-86, :152-153). */
typedef struct vp3d_cfg {
    int32_t num_joints_in;
    int32_t in_features;
    int32_t num_joints_out;
    int32_t n_widths;                        /* len(filter_widths)                  */
    int32_t filter_widths[VP3D_MAX_BLOCKS];  /* odd widths, e.g. 3,3,3,3,3          */
    int32_t causal;                          /* 0/1                                 */
    int32_t channels;                        /* e.g. 1024                           */
    int32_t dense;                           /* 0/1 (dilated variant only)          */
    int32_t variant;                         /* VP3D_VARIANT_*                      */
    float bn_eps;                            /* BatchNorm1d eps (1e-5 in reference) */
} vp3d_cfg;

typedef struct vp3d_handle vp3d_handle;

/* ---- lifecycle (replaces TemporalModel.__init__ + load_state_dict + .cuda()) ---- */

/* Number of host weight arrays vp3d_create / vp3d_load_weights expect, in
 * state_dict order (TemporalModel.py:32-33,102,113-119):
 *   expand_conv.weight (C, J_in*F, w0)
 *   expand_bn.{weight, bias, running_mean, running_var} (C each)
 *   for i in 0..2*(n_widths-1)-1:
 *       layers_conv.i.weight (C, C, k_i)
 *       layers_bn.i.{weight, bias, running_mean, running_var}
 *   shrink.weight (J_out*3, C, 1), shrink.bias (J_out*3)
 * i.e. 5 + 10*(n_widths-1) + 2 arrays of float32, contiguous, PyTorch layout.
 * Returns the count, or -1 on an invalid configuration. */
int vp3d_weight_count(const vp3d_cfg* cfg);

/* Validate cfg (odd widths: TemporalModel.py:20-21), fold every eval-mode
 * BatchNorm into a per-channel (scale, shift) pair, pack the convolution
 * weights tap-major for the MFMA kernels (f32 and bf16 copies) and upload them
 * to the current HIP device.  `weights` are HOST pointers. */
int vp3d_create(const vp3d_cfg* cfg, const float* const* weights, int n_weights, vp3d_handle** out);

/* Re-pack and re-upload weights into an existing handle (load_state_dict,
 * TemporalModel.py via nn.Module; called by run.py:416-417). Synchronous. */
int vp3d_load_weights(vp3d_handle* h, const float* const* weights, int n_weights);

int vp3d_destroy(vp3d_handle* h);

/* ---- shape helpers (TemporalModel.py:40-60) ---- */
int vp3d_receptive_field(const vp3d_handle* h);     /* 1 + 2*sum(pad)               */
int vp3d_total_causal_shift(const vp3d_handle* h);  /* bit-compatible, quirk Q5     */
/* Output frames for an input of T frames, or -1 if T is invalid for the variant. */
int vp3d_out_frames(const vp3d_handle* h, int T);

/* ---- forward (replaces TemporalModelBase.forward, TemporalModel.py:62-76) ---- */

/* Allocate the activation workspace for (B, T, dtype) up front so that a later
 * vp3d_forward with B' <= B, T' <= T allocates nothing (and can be captured into
 * a hipGraph). */
int vp3d_reserve(vp3d_handle* h, int B, int T, int dtype);

/* Eval-mode forward.  x: device f32 (B, T, J_in, F) contiguous.
 * y: device f32 (B, vp3d_out_frames(T), J_out, 3) contiguous, written here.
 * Launches on `stream`; returns without synchronising. */
int vp3d_forward(vp3d_handle* h, const float* x, int B, int T, float* y, int dtype, void* stream);

/* Synchronise `stream` and report a device-side fault of this handle's launches since the
 * last call: VP3D_ERR_STATE when a split-K owner tile (conv_gemm_a4, the partial last round
 * of small f16x3 batches) gave up waiting for its helper units -- its output was then
 * wrong -- or when an f16x3 forward split a value past the f16 range of its halves
 * (|x| > 65,504: checked where the input rows and every hidden activation are split) or
 * produced non-finite poses (run such inputs in fp32); the fault is cleared by this call.  (The next vp3d_forward* on the handle also
 * refuses with VP3D_ERR_STATE while the fault is pending, without synchronising -- every
 * dtype after a split-K timeout, f16x3 only after an f16x3 range fault.)  No
 * reference counterpart: torch raises asynchronous device errors at the next sync. */
int vp3d_sync_status(vp3d_handle* h, void* stream);

/* Eval-mode forward of B windows gathered on the fly from device-resident
 * sequences: the ChunkedGenerator batch (generators.py:102-137; edge padding of
 * pad_chunk :92-100) and the trajectory concat (CamTransformer.py:187-190) feeding
 * TemporalModelBase.forward (TemporalModel.py:62-76) without materialising the
 * (B, window, J_in*F) input.  On the 16-bit path the gather is fused into the
 * expand conv's operand loads; otherwise the windows go through a scratch tensor.
 *   kps:     device f32 (n_frames, f2) normalised keypoints of all sequences
 *   cams:    device f32 (n_frames, 12) per-frame K.E, or NULL (no concat);
 *            f2 (+ 12) must equal num_joints_in * in_features
 *   seq_off: device int64 first frame of each sequence; seq_len: device int32
 *   pairs:   device int32 (B, 2) = (sequence, start); window b = sequence frames
 *            [start - lead, start - lead + window), clamped to [0, len-1]
 *   y:       device f32 (B, vp3d_out_frames(window), J_out, 3)
 * With cams, dtype VP3D_DTYPE_BF16 is refused (VP3D_ERR_ARG): its 8-bit mantissa on the
 * metre-scale K.E channels costs ~30 mm; fp16, f16x3 (the accurate fast path) or f32. */
int vp3d_forward_windows(vp3d_handle* h, const float* kps, int32_t f2, const float* cams,
                         const int64_t* seq_off, const int32_t* seq_len, const int32_t* pairs, int B,
                         int window, int lead, float* y, int dtype, void* stream);

/* ---- per-layer timing (HIP events recorded on the launch stream) ---- */
int vp3d_profile_enable(vp3d_handle* h, int enable);
/* Restrict the timing to the layers in `mask` (bit i = layer i; all by default), e.g.
 * only the dominant layer inside a timed loop so the other launches carry no events. */
int vp3d_profile_layers(vp3d_handle* h, uint64_t mask);
/* Number of kernel launches one forward makes (conv layers incl. shrink). */
int vp3d_layer_count(const vp3d_handle* h);
/* Accumulated time (ms) and launch count per layer since the last reset, and
 * the algorithmic FLOP of each layer's most recent launch.  Synchronises on
 * the recorded events.  Arrays have vp3d_layer_count() entries. */
int vp3d_profile_read(vp3d_handle* h, double* ms_total, int64_t* launches, double* flop_last);
int vp3d_profile_reset(vp3d_handle* h);

/* ---- causal streaming (BASELINE config 5) ----
 * One frame in, one pose out, for a causal dilated model (TemporalModel with
 * causal=True, TemporalModel.py:107-111): every convolution is a GEMV over taps
 * read from per-layer ring buffers of past activations.  Output k equals frame k
 * of the reference's whole-sequence causal evaluation (UnchunkedGenerator edge
 * padding, generators.py:193-198).  The stream position lives in device memory,
 * so one step is replayable from a hipGraph. */
typedef struct vp3d_stream vp3d_stream;

/* dtype: VP3D_DTYPE_* of the weights streamed per step (f16 in config 5; F32 keeps the
 * exact fp32 weights resident, the north-star accuracy form). */
int vp3d_stream_create(vp3d_handle* h, int dtype, vp3d_stream** out);
/* Restart the stream (the next frame is frame 0).  Async on `stream`. */
int vp3d_stream_reset(vp3d_stream* s, void* stream);
/* Device frame queue and pose ring of the stream (queue_len slots each, a power of
 * two): step t reads frame slot t % queue_len and writes pose slot t % queue_len.
 * Graph replays read/write exactly these; frames can be queued ahead of time. */
int vp3d_stream_io(vp3d_stream* s, float** in_frames, float** out_poses, int* queue_len);
/* One step.  frame / pose: device pointers (frame copied into the queue slot of
 * this step, pose copied out of it, asynchronously), or NULL to use the queue
 * slot as is. */
int vp3d_stream_step(vp3d_stream* s, const float* frame, float* pose, void* stream);
/* Frames consumed so far (synchronises with the device). */
int64_t vp3d_stream_frames_seen(vp3d_stream* s);
/* Capture `steps` consecutive steps (frames from the queue) into a hipGraph on
 * `stream` (not the legacy default stream); replay with vp3d_stream_graph_launch. */
int vp3d_stream_graph_capture(vp3d_stream* s, void* stream, int steps);
int vp3d_stream_graph_launch(vp3d_stream* s, void* stream);
int vp3d_stream_destroy(vp3d_stream* s);
/* 1 when the stream runs as one persistent launch per batch of steps (weights resident
 * on chip, layer outputs handed between CUs in-launch), 0 for one GEMV launch per layer
 * (VP3D_STREAM_MODE=launches at vp3d_stream_create, or a shape no persistent form takes). */
int vp3d_stream_persistent(const vp3d_stream* s);
/* Form of the in-launch step: 2 = layer-pipelined (stream_pipe.hip: each CU runs one
 * layer with its weights in VGPRs, frames of a batch pipelined through the layer groups;
 * the default at 1024 / 256 channels with 3-tap blocks, f32 weights held as they are,
 * 16-bit ones widened to f32), 1 = every CU runs every layer with its 16-bit weights in LDS
 * (stream_persist.hip), 0 = one GEMV launch per layer.  VP3D_STREAM_MODE=pipe|persist|launches at vp3d_stream_create restricts it. */
int vp3d_stream_mode(const vp3d_stream* s);
/* Synchronises; VP3D_ERR_STATE if a persistent launch gave up waiting on another CU
 * (bounded spins: the grid did not fit the device at once), else VP3D_OK. */
int vp3d_stream_status(vp3d_stream* s);

/* ---- serving: one frame in flight, real time (config 5's single-frame latency) ----
 * The layer-pipelined launch (mode 2) stays resident with its weights in VGPRs and takes
 * frames as the host posts them through pinned host memory; the pose of frame t comes back
 * the same way, with no launch, copy or graph per frame.  The launch ends by itself at
 * the first frame not posted within idle_ms, or at vp3d_stream_serve_end.  Frames keep
 * the stream's numbering (the first posted frame is frame vp3d_stream_frames_seen()).
 * At most queue_len - 1 frames may be posted and not yet waited for.
 * The last block's 1x1 workgroups fold the shrink in (VP3D_STREAM_FOLD, default on): each
 * stores its channels' partial pose sums and the host adds them in a fixed order (one layer
 * group fewer on the frame's path: median 24.4 vs 25.4 us), so served poses equal the batch
 * form's within 1e-6 m, not bit for bit; the host-side shrink affine is re-read from the
 * handle at every serve_begin (after vp3d_load_weights too).  hipFree / hipDeviceSynchronize anywhere in the
 * process wait for the resident launch (it ends at idle_ms): end serving before freeing
 * device memory or destroying another stream.
 */
int vp3d_stream_serve_begin(vp3d_stream* s, void* stream, double idle_ms);
/* Copy one frame (host f32, J_in * F values) into the ring and post it; *frame_index is
 * its stream index.  VP3D_ERR_STATE when not serving, the ring is full or the launch ended. */
int vp3d_stream_serve_post(vp3d_stream* s, const float* frame, int64_t* frame_index);
/* Wait (spinning on host memory, at most timeout_ms) until frame `frame_index` is done and
 * copy its pose (host f32, J_out * 3) out.  VP3D_ERR_STATE on timeout or stream fault. */
int vp3d_stream_serve_wait(vp3d_stream* s, int64_t frame_index, float* pose, double timeout_ms);
/* post + wait in one call (one frame in flight); *latency_us (or NULL) = host wall time from
 * the start of the post to the pose copied out. */
int vp3d_stream_serve_step(vp3d_stream* s, const float* frame, float* pose, double timeout_ms, double* latency_us);
/* Stop serving: the launch finishes the posted frames and exits; synchronises `stream`. */
int vp3d_stream_serve_end(vp3d_stream* s, void* stream);
/* Diagnostics of the layer-pipelined form (no reference counterpart): with VP3D_STREAM_TRACE=n
 * set at vp3d_stream_create, every workgroup records the 100 MHz device clock when the input of
 * each of the first n frames of a launch is complete and, per wave, after the wave's first
 * output store.  Copies workgroups x n x 11 clocks ([0] input complete, [1 + w] wave w stored;
 * [9], [10]: the shader clock counter at [0] and [1]) to `out` (NULL: sizes only) and clears them; role_first_wg (n_roles
 * + 1 entries, or NULL) = the first workgroup of each layer role (expand, k / 1x1 per block,
 * shrink).  Synchronises the device. */
int vp3d_stream_trace(vp3d_stream* s, uint64_t* out, int64_t capacity, int32_t* role_first_wg, int32_t* n_roles,
                      int32_t* frames);

/* ---- training step (run.py:451-487, :662) ----
 * The reference trains TemporalModel in train mode: BatchNorm1d on batch
 * statistics with a running-stat update (TemporalModel.py:117,119; momentum
 * decayed per epoch by set_bn_momentum :35-38, run.py:553-556), ReLU, Dropout
 * (:130-137), the residual add, then loss.backward() and
 * optim.Adam(amsgrad=True).step().  A trainer runs that forward/backward on the
 * device in f32.  Parameters stay in caller-owned device memory (the
 * nn.Module's own tensors) and are passed per call as a table of device
 * pointers in state_dict order — the same order and count as vp3d_create's
 * `weights` (vp3d_weight_count): conv weight, then BN weight / bias /
 * running_mean / running_var per conv, shrink weight and bias.  Dropout masks
 * come from a counter-based hash of (seed, layer, element), regenerated in the
 * backward rather than stored (vp3d_train_dropout_mask exports them). */
typedef struct vp3d_trainer vp3d_trainer;

int vp3d_trainer_create(const vp3d_cfg* cfg, vp3d_trainer** out);
int vp3d_trainer_destroy(vp3d_trainer* t);

/* Train-mode forward (TemporalModelBase.forward in train mode, TemporalModel.py:62-76).
 * params: host array of n_params DEVICE pointers (state_dict order); the BN
 * running_mean / running_var entries are updated in place with `momentum`
 * (BatchNorm1d.momentum).  x: device f32 (B, T, J_in, F); y: device f32
 * (B, vp3d_out_frames(T), J_out, 3).  dropout_p: nn.Dropout p; seed: mask seed.
 * The activations the backward needs are kept inside the trainer until the next
 * forward. */
int vp3d_train_forward(vp3d_trainer* t, float* const* params, int n_params, const float* x, int B, int T,
                       float dropout_p, double momentum, uint64_t seed, float* y, void* stream);

/* Backward of the latest vp3d_train_forward (same params, which must not have
 * changed in between).  dy: device f32 like y.  grads: host array of n_params
 * device pointers, state_dict order; each trainable entry receives its gradient
 * (overwritten, torch layout); running-stat entries are ignored and may be NULL.
 * The input gradient is not formed (the 2D keypoints are data, run.py:458). */
int vp3d_train_backward(vp3d_trainer* t, float* const* params, int n_params, const float* dy,
                        float* const* grads, void* stream);

/* The dropout keep mask (1 = kept) of conv layer `layer` (0 = expand, then the
 * block convs in order) for the latest forward: n_elems = rows * channels of that
 * layer's output, row-major (b, t, c).  Test hook for the parity tests. */
int vp3d_train_dropout_mask(vp3d_trainer* t, int layer, int64_t n_elems, uint8_t* out, void* stream);

/* The ReLU mask (1 = BN output > 0) of conv layer `layer` in the latest forward, same
 * layout as vp3d_train_dropout_mask.  Test hook: an element whose BN output lies within
 * rounding of 0 may take the other side of the ReLU in another f32 implementation, so the
 * parity tests feed this mask (with the dropout mask) to the oracle. */
int vp3d_train_relu_mask(vp3d_trainer* t, int layer, int64_t n_elems, uint8_t* out, void* stream);

/* Row count (B * frames) of conv layer `layer`'s output in the latest forward, or -1. */
int64_t vp3d_train_layer_rows(const vp3d_trainer* t, int layer);

/* One Adam step over n tensors (torch.optim.Adam, _single_tensor_adam; run.py:662
 * builds it with amsgrad=True): for each i, with g = grad (+ weight_decay * param),
 *   exp_avg = lerp(exp_avg, g, 1 - beta1)   (as fma, like ATen's vectorised lerp)
 *   exp_avg_sq = fma((1 - beta2) * g, g, exp_avg_sq * beta2)
 *   max_exp_avg_sq = max(max_exp_avg_sq, exp_avg_sq)                    (amsgrad)
 *   param += -lr / (1 - beta1^step) * exp_avg / (sqrt(max_exp_avg_sq or exp_avg_sq)
 *                                                / sqrt(1 - beta2^step) + eps)
 * `step` is the already-incremented step count.  All arrays are host arrays of
 * device pointers / element counts; max_exp_avg_sq entries may be NULL without
 * amsgrad.  n <= 64 per call. */
int vp3d_adam_step(int n, float* const* params, const float* const* grads, float* const* exp_avg,
                   float* const* exp_avg_sq, float* const* max_exp_avg_sq, const int64_t* numel, double lr,
                   double beta1, double beta2, double eps, double weight_decay, int64_t step, int amsgrad,
                   void* stream);

/* ---- trajectory-conditioned sequence lifters, eval mode ----
 * CoupledTransformer (common/models/CamTransformer.py:95-205) and CoupledLSTM
 * (common/models/CamLSTM.py:47-129): per frame [flat 2D | flat K.E] (:187-190 /
 * :115-121), then a transformer encoder or a stacked LSTM over a window, the last
 * step through an MLP head.  f32. */
#define VP3D_SEQ_TRANSFORMER 0
#define VP3D_SEQ_LSTM 1
#define VP3D_SEQ_MAX_HEAD 8

typedef struct vp3d_seq_cfg {
    int32_t kind;            /* VP3D_SEQ_*                                                 */
    int32_t num_joints_in, in_features, num_joints_out, out_features;
    int32_t d_model;         /* transformer d_model / LSTM hidden_size                     */
    int32_t num_layers;      /* encoder layers / LSTM cells (<= 4)                         */
    int32_t n_heads;         /* transformer only; d_model / n_heads in {16, 32, 64}        */
    int32_t dim_feedforward; /* transformer only                                           */
    int32_t n_head_layers;   /* len(head_layers)                                           */
    int32_t head_layers[VP3D_SEQ_MAX_HEAD];
    int32_t max_len;         /* rows of the positional-encoding table (5000)               */
    float eps;               /* LayerNorm / BatchNorm eps (1e-5)                           */
} vp3d_seq_cfg;

typedef struct vp3d_seq_lifter vp3d_seq_lifter;

/* Host weight arrays vp3d_seq_create expects, in state_dict order without the
 * BatchNorm num_batches_tracked counters:
 *   transformer: input_projection.{weight, bias}, positional_encoding.pe (max_len x d),
 *     pre_transformer_norm.{weight, bias}, per encoder layer self_attn.in_proj_{weight, bias},
 *     self_attn.out_proj.{weight, bias}, linear1.{weight, bias}, linear2.{weight, bias},
 *     norm1.{weight, bias}, norm2.{weight, bias}; mlp_layers Linear {weight, bias} x (heads + 1)
 *   lstm: per cell weight_ih, weight_hh, bias_ih, bias_hh; bn_lstm.{weight, bias,
 *     running_mean, running_var}; per head layer Linear {weight, bias} + BatchNorm1d
 *     {weight, bias, running_mean, running_var}; the last Linear {weight, bias}
 * Returns the count, or -1 for an invalid configuration. */
int vp3d_seq_weight_count(const vp3d_seq_cfg* cfg);
int vp3d_seq_create(const vp3d_seq_cfg* cfg, const float* const* weights, int n_weights, vp3d_seq_lifter** out);
int vp3d_seq_destroy(vp3d_seq_lifter* h);

/* forward(input_2d, input_cam) (CamTransformer.py:165-205, CamLSTM.py:104-129):
 * x2d device f32 (B, T, J_in, F), xcam device f32 (B, T, 3, 4) -> y device f32
 * (B, 1, J_out, out_features). */
int vp3d_seq_forward(vp3d_seq_lifter* h, const float* x2d, const float* xcam, int B, int T, float* y, void* stream);

/* sliding_window(inputs_2d, inputs_cam, window) (CamTransformer.py:72-92): x2d (L, J_in, F),
 * xcam (L, 3, 4) of one sequence -> y (L - window + 1, J_out, out_features), window w =
 * frames [w, w + window).  The per-frame input projection is shared by all windows; no
 * (n_windows, window, ...) copy is made. */
int vp3d_seq_sliding_window(vp3d_seq_lifter* h, const float* x2d, const float* xcam, int L, int window, float* y,
                            void* stream);

/* ---- on-device input path (common/camera.py, common/generators.py) ---- */

/* normalize_screen_coordinates (camera.py:14-18): out = X/w*2 - [1, h/w] for
 * n_points (x, y) pairs, with the reference's float64 promotion of the offset
 * reproduced exactly (quirk Q6).  Device pointers, in-place allowed. */
int vp3d_normalize_screen(const float* x, int64_t n_points, int32_t w, int32_t h, float* out,
                          void* stream);

/* normalize_screen_coordinates on float64 keypoints with a non-integral resolution (the
 * 3DPW path: keypoints stored f64, w = 2 c_x a float32 scalar, run.py:117 /
 * ThreeDPWDataset.py:87-103): out = f32(X/w*2 - [1, hw]) with the whole expression in
 * float64, i.e. the reference's float64 result rounded once when its generator casts the
 * batch (run.py:458).  hw = the value h / w takes in the caller's arithmetic (float32
 * division for float32 w, h). */
int vp3d_normalize_screen_f64(const double* x, int64_t n_points, double w, double hw, float* out,
                              void* stream);

/* image_coordinates (camera.py:21-25): out = (X + [1, h/w]) * w / 2. */
int vp3d_image_coordinates(const float* x, int64_t n_points, int32_t w, int32_t h, float* out,
                           void* stream);

/* Per-frame camera matrices K @ E_t (generators.py:115-125, :180-190).
 * intr: device f32 [fx, fy, cx, cy] per sequence (n_seq x 4); frame_seq: device
 * int32 sequence id of each frame; extr: device f64 (n_frames, 3, 4) extrinsics;
 * out: device f32 (n_frames, 12).  Evaluated in float64 like the reference's
 * float32 @ float64 numpy matmul, then rounded once to f32. */
int vp3d_camera_matrices(const float* intr, const int32_t* frame_seq, const double* extr,
                         int64_t n_frames, float* out, void* stream);

/* world_to_camera (camera.py:28-30 -> quaternion.py:10-35):
 * out = qrot(qinverse(R), X - t) for n_points 3-vectors; R (4,) and t (3,) host
 * values (one camera per call, like the reference). */
int vp3d_world_to_camera(const float* X, int64_t n_points, const float* R_host,
                         const float* t_host, float* out, void* stream);

/* Window gather with edge padding (ChunkedGenerator.pad_chunk/next_epoch,
 * generators.py:92-137; UnchunkedGenerator edge pad :193-198), fused with the
 * trajectory concat (CamTransformer.py:187-190).
 *   kps:      device f32 (n_frames, F2) normalised 2D keypoints (F2 = J*2)
 *   cams:     device f32 (n_frames, 12) camera matrices or NULL (no concat)
 *   seq_off:  device int64 first frame of each sequence; seq_len: device int32
 *   pairs:    device int32 (B, 2) = (sequence id, first output frame start_3d)
 *   out:      device f32 (B, window, F2 [+12])
 * Window b covers frames [start_3d - pad - shift, start_3d - pad - shift + window)
 * of its sequence, indices clamped to [0, len-1] ('edge' padding). */
int vp3d_gather_windows(const float* kps, int32_t f2, const float* cams, const int64_t* seq_off,
                        const int32_t* seq_len, const int32_t* pairs, int32_t B, int32_t window,
                        int32_t pad, int32_t causal_shift, float* out, void* stream);

/* project_to_2d (camera.py:37-67: H36M radial + tangential distortion) or, with
 * linear != 0, project_to_2d_linear (:69-90): X device f32 (n_cams, pts_per_cam, 3)
 * camera-space points, params device f32 (n_cams, 9) = [f(2), c(2), k(3), p(2)],
 * out device f32 (n_cams, pts_per_cam, 2).  Same float32 operation order as the
 * reference's torch code (bit-exact on the goldens). */
int vp3d_project_to_2d(const float* X, int64_t n_cams, int64_t pts_per_cam, const float* params,
                       int32_t linear, float* out, void* stream);

/* mpjpe partial sums (loss.py:11-17): acc[0] += sum ||pred - target||_2 over
 * n_points xyz triples, acc[1] += n_points.  acc: device f64[2] (caller zeroes). */
int vp3d_mpjpe_accumulate(const float* pred, const float* target, int64_t n_points, double* acc,
                          void* stream);

/* Gradient of the training loss mpjpe = mean ||pred - target|| (loss.py:11-17, run.py:478)
 * with respect to pred: grad_pred = grad_loss[0] / n_points * (pred - target) / ||pred - target||
 * per point (0 where the distance is 0).  grad_loss: device f32 scalar (the upstream
 * gradient, 1 for loss.backward()); grad_pred: device f32 like pred. */
int vp3d_mpjpe_backward(const float* pred, const float* target, int64_t n_points, const float* grad_loss,
                        float* grad_pred, void* stream);

/* Evaluation metrics of one sequence's predictions (run.py:732-750): partial sums of
 * MPJPE (loss.py:11-17), P-MPJPE (rigid alignment per frame, loss.py:29-68), N-MPJPE
 * (per-frame scale, loss.py:70-80) and MPJVE (first difference along frames,
 * loss.py:82-91) over pred / target (n_frames, n_joints, 3), float64:
 *   acc[0..3] += summed per-joint errors (MPJPE, P-MPJPE, N-MPJPE, MPJVE)
 *   acc[4] += n_frames * n_joints,  acc[5] += (n_frames - 1) * n_joints
 * acc: device f64[6] (caller zeroes).  Metric = acc[i] / acc[4] (i < 3), acc[3] / acc[5]. */
int vp3d_pose_metrics(const float* pred, const float* target, int64_t n_frames, int32_t n_joints,
                      double* acc, void* stream);

const char* vp3d_last_error(void);
int vp3d_abi_version(void);
/* SHA-256 (hex) of the sources this library was built from: every csrc/ translation unit
 * and header plus include/vp3d.h and the compiler flags (vp3d_amd/build.py source_hash).
 * The Python loader refuses a library whose hash differs from the tree beside it. */
const char* vp3d_build_hash(void);

#ifdef __cplusplus
}
#endif

#endif /* VP3D_H */
