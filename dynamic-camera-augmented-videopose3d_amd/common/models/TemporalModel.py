"""Drop-in replacement for the reference's ``common/models/TemporalModel.py``.

Same public classes, constructor signatures, attributes (``pad``,
``causal_shift``, ``filter_widths``, ``expand_conv``, ``expand_bn``,
``layers_conv``, ``layers_bn``, ``shrink``, ``drop``, ``relu``), methods and
state_dict keys as Bart-Weil/Dynamic-Camera-Augmented-VideoPose3D
common/models/TemporalModel.py:

  TemporalModelBase         :10-76   receptive_field :40-47, total_causal_shift :49-60,
                                     set_bn_momentum :35-38, forward :62-76
  TemporalModel             :79-138  dilated convolutions (and the dense ablation)
  TemporalModelOptimized1f  :141-198 strided single-frame twin, interchangeable weights

Eval-mode forward on a HIP device runs the MI355X kernels of libvp3d.so
(include/vp3d.h ``vp3d_forward``): every convolution is one MFMA GEMM whose
epilogue applies the folded BatchNorm, ReLU, dropout (identity in eval) and the
residual slice-add.  A CPU input in eval mode raises — there is no fallback.

Train mode runs the native training step too
(include/vp3d.h ``vp3d_train_forward`` / ``vp3d_train_backward`` through the
autograd node ``vp3d_amd.train.TrainStep``): BatchNorm batch statistics with the
running-stat update, ReLU, dropout (counter-hash masks), the residual add and the
backward of every layer, all in f32 on the device, so the reference's training loop
(``loss.backward()``, ``optimizer.step()``) runs unchanged.  A CPU input raises in
train mode as in eval mode.

Precision: fp32 by default (exact f32 MFMA, the parity path);
``model.set_compute_dtype('bf16' | 'fp16')`` selects the 16-bit MFMA path.
"""
import torch
import torch.nn as nn

from vp3d_amd import _native as _N
from vp3d_amd.lifter import NativeLifter, weight_order
from vp3d_amd.train import NativeTrainer, TrainStep

__all__ = ["TemporalModelBase", "TemporalModel", "TemporalModelOptimized1f"]


def _plan_blocks(filter_widths, causal, strided, dense):
    """Per-block geometry shared by construction and the train-mode graph.

    Returns (pad, causal_shift, blocks) where ``blocks[i]`` describes the
    (k-conv, 1x1-conv) pair of block i+1: kernel size, dilation, stride and the
    residual slice (start, step) taken from the block input."""
    w0 = filter_widths[0]
    pad = [w0 // 2]
    shift = [w0 // 2 if causal else 0]
    blocks = []
    dilation = w0
    for w in filter_widths[1:]:
        p = (w - 1) * dilation // 2
        pad.append(p)
        if strided:
            s = w // 2 if causal else 0                     # not dilation-scaled (:177)
            blocks.append(dict(kernel=w, dilation=1, stride=w, res_start=s + w // 2, res_step=w))
        else:
            s = (w // 2) * dilation if causal else 0        # dilation-scaled (:111)
            kernel, dil = (2 * p + 1, 1) if dense else (w, dilation)
            blocks.append(dict(kernel=kernel, dilation=dil, stride=1, res_start=p + s,
                               res_trim=p - s, res_step=1))
        shift.append(s)
        dilation *= w
    return pad, shift, blocks


class TemporalModelBase(nn.Module):
    """Shared state of the two lifter variants (not meant to be instantiated)."""

    _variant = None  # VARIANT_DILATED / VARIANT_STRIDED_1F, set by subclasses

    def __init__(self, num_joints_in, in_features, num_joints_out,
                 filter_widths, causal, dropout, channels):
        super().__init__()
        for fw in filter_widths:
            assert fw % 2 != 0, 'Only odd filter widths are supported'

        self.num_joints_in = num_joints_in
        self.in_features = in_features
        self.num_joints_out = num_joints_out
        self.filter_widths = filter_widths
        self.causal = causal
        self.channels = channels
        self.dense = False

        self.drop = nn.Dropout(dropout)
        self.relu = nn.ReLU(inplace=True)
        self.pad = [filter_widths[0] // 2]
        self.expand_bn = nn.BatchNorm1d(channels, momentum=0.1)
        self.shrink = nn.Conv1d(channels, num_joints_out * 3, 1)

        self.compute_dtype = 'fp32'
        self._lifter = None
        self._lifter_key = None
        self._trainer = None

    def _build_stack(self, strided, dense):
        pad, shift, blocks = _plan_blocks(self.filter_widths, self.causal, strided, dense)
        self.pad = pad
        self.causal_shift = shift
        self._blocks = blocks
        c = self.channels
        w0 = self.filter_widths[0]
        self.expand_conv = nn.Conv1d(self.num_joints_in * self.in_features, c, w0,
                                     stride=w0 if strided else 1, bias=False)
        convs, bns = [], []
        for blk in blocks:
            convs.append(nn.Conv1d(c, c, blk["kernel"], stride=blk["stride"],
                                   dilation=blk["dilation"], bias=False))
            bns.append(nn.BatchNorm1d(c, momentum=0.1))
            convs.append(nn.Conv1d(c, c, 1, dilation=1, bias=False))
            bns.append(nn.BatchNorm1d(c, momentum=0.1))
        self.layers_conv = nn.ModuleList(convs)
        self.layers_bn = nn.ModuleList(bns)

    # ---- reference API -------------------------------------------------------------
    def set_bn_momentum(self, momentum):
        for bn in [self.expand_bn, *self.layers_bn]:
            bn.momentum = momentum

    def receptive_field(self):
        """Frames of context one output frame sees: 1 + 2 * sum(pad)."""
        return 1 + 2 * sum(self.pad)

    def total_causal_shift(self):
        """The reference's asymmetric-padding offset, reproduced bit for bit —
        including its second dilation scaling of the dilated variant's
        already-scaled shifts.  run.py uses ``pad`` instead."""
        total, dilation = self.causal_shift[0], self.filter_widths[0]
        for w, s in zip(self.filter_widths[1:], self.causal_shift[1:]):
            total += s * dilation
            dilation *= w
        return total

    def set_compute_dtype(self, dtype):
        """'fp32' (default, parity path), 'f16x3' (split fp16: fp32-level results on the 16-bit
        MFMAs), 'bf16' or 'fp16'."""
        if dtype not in _N.DTYPES:
            raise ValueError(f"unknown compute dtype {dtype!r}")
        self.compute_dtype = dtype
        return self

    # ---- native engine -------------------------------------------------------------
    def _state_signature(self, device):
        sig = [str(device)]
        for t in self.state_dict(keep_vars=True).values():
            sig.append((t.data_ptr(), t._version))
        return tuple(sig)

    def native_lifter(self, device=None) -> NativeLifter:
        """The NativeLifter holding this module's folded weights on `device`;
        re-packed whenever a parameter or buffer was replaced or modified."""
        device = torch.device(device if device is not None else self.expand_conv.weight.device)
        if device.type != 'cuda':
            raise RuntimeError(
                "vp3d: the eval-mode lifter runs on the MI355X kernels only; move the model "
                "and inputs to the GPU with .cuda() (no CPU fallback)")
        key = self._state_signature(device)
        if self._lifter is not None and self._lifter_key == key:
            return self._lifter
        state = dict(self.state_dict())
        if self._lifter is not None and self._lifter.device == device:
            self._lifter.load_weights(state)
        else:
            self._lifter = NativeLifter(self.num_joints_in, self.in_features, self.num_joints_out,
                                        self.filter_widths, self.causal, self.channels,
                                        self.dense, self._variant, state, device=device,
                                        bn_eps=self.expand_bn.eps)
        self._lifter_key = key
        return self._lifter

    def sync_status(self):
        """Synchronise and raise RuntimeError if an eval-mode forward of this module reported a
        device-side fault that has not been raised yet (NativeLifter.sync_status: a split-K
        timeout, or an f16x3 activation past the f16 range / non-finite poses).  A forward
        raises a pending fault of an EARLIER forward at entry; the last forward of a run is
        only checked here (vp3d_amd.evaluate.evaluate calls it after its loop).  No-op
        before the first eval-mode forward."""
        if self._lifter is not None:
            self._lifter.sync_status()

    def native_trainer(self, device) -> NativeTrainer:
        """The NativeTrainer (train-mode forward/backward engine) for `device`."""
        device = torch.device(device)
        if self._trainer is None or self._trainer.device != device:
            self._trainer = NativeTrainer(self.num_joints_in, self.in_features, self.num_joints_out,
                                          self.filter_widths, self.causal, self.channels, self.dense,
                                          self._variant, device, bn_eps=self.expand_bn.eps)
        return self._trainer

    def forward(self, x):
        """TemporalModel.py:62-76.  Eval mode runs libvp3d (compute dtype: set_compute_dtype);
        a device-side fault of an EARLIER eval forward (split-K timeout; f16x3 range, which
        blocks only f16x3 forwards) raises RuntimeError here, and one of the last forward is
        raised by sync_status() -- call it before trusting a run's final outputs."""
        assert len(x.shape) == 4
        assert x.shape[-2] == self.num_joints_in
        assert x.shape[-1] == self.in_features
        if not x.is_cuda:
            raise RuntimeError(
                "vp3d: the lifter runs on the MI355X kernels only (no CPU fallback); "
                "call model.cuda() and pass x.cuda()")
        if self.training:
            return self._train_forward(x)
        return self.native_lifter(x.device).forward(x, self.compute_dtype)

    def _train_forward(self, x):
        """Train-mode forward through the native trainer (TemporalModel.py:62-76, :126-138 /
        :188-198 with BatchNorm1d in training mode and nn.Dropout active)."""
        bns = [self.expand_bn, *self.layers_bn]
        momentum = bns[0].momentum
        if any(bn.momentum != momentum for bn in bns):
            raise NotImplementedError("vp3d: per-layer BatchNorm momenta differ (set_bn_momentum sets one)")
        if any(not bn.track_running_stats or not bn.training for bn in bns):
            raise NotImplementedError("vp3d: train mode needs every BatchNorm training with running stats")
        # BatchNorm1d.forward: count the batch; cumulative average when momentum is None
        for bn in bns:
            bn.num_batches_tracked.add_(1)
        factor = (1.0 / float(bns[0].num_batches_tracked.item())) if momentum is None else momentum
        state = self.state_dict(keep_vars=True)
        tensors = [state[k] for k in weight_order(len(self.filter_widths))]
        for t in tensors:
            if t.device != x.device or t.dtype != torch.float32 or not t.is_contiguous():
                raise RuntimeError("vp3d: parameters must be contiguous float32 tensors on the input's device")
        trainable = tuple(isinstance(t, nn.Parameter) and t.requires_grad for t in tensors)
        trainer = self.native_trainer(x.device)
        T_out = self._out_frames(int(x.shape[1]))
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if self.drop.p > 0 else 0
        x = x.contiguous().float()
        return TrainStep.apply(trainer, float(self.drop.p), float(factor), seed, T_out, trainable, x, *tensors)

    def _out_frames(self, T):
        """Output frames for T input frames (the conv length rules of TemporalModel.py)."""
        w0 = self.filter_widths[0]
        strided = self._variant == _N.VARIANT_STRIDED_1F
        L = (T - w0) // w0 + 1 if strided else T - (w0 - 1)
        for blk in self._blocks:
            span = (blk["kernel"] - 1) * blk["dilation"] + 1
            L = (L - span) // blk["stride"] + 1 if L >= span else 0
        if L < 1:
            raise RuntimeError(f"input of {T} frames is shorter than the receptive field "
                               f"{self.receptive_field()}")
        return L


class TemporalModel(TemporalModelBase):
    """Dilated temporal-convolution lifter: any T >= receptive_field() frames in,
    T - receptive_field() + 1 poses out (reference TemporalModel.py:79-138)."""

    _variant = _N.VARIANT_DILATED

    def __init__(self, num_joints_in, in_features, num_joints_out,
                 filter_widths, causal=False, dropout=0.25, channels=1024, dense=False):
        super().__init__(num_joints_in, in_features, num_joints_out, filter_widths, causal,
                         dropout, channels)
        self.dense = dense
        self._build_stack(strided=False, dense=dense)


class TemporalModelOptimized1f(TemporalModelBase):
    """Strided single-frame lifter: windows of receptive_field() frames in, one pose
    out; weights interchangeable with TemporalModel (reference TemporalModel.py:141-198)."""

    _variant = _N.VARIANT_STRIDED_1F

    def __init__(self, num_joints_in, in_features, num_joints_out,
                 filter_widths, causal=False, dropout=0.25, channels=1024):
        super().__init__(num_joints_in, in_features, num_joints_out, filter_widths, causal,
                         dropout, channels)
        self._build_stack(strided=True, dense=False)
