"""ORACLE (test infrastructure only): CPU restatement of one training iteration.

Follows the reference's training loop run.py:451-487 around TemporalModel in train
mode (common/models/TemporalModel.py:62-76, :126-138, :188-198):

  forward    drop(relu(bn(conv(x)))) per conv, BatchNorm1d on batch statistics with
             the running-stat update (momentum, TemporalModel.py:32,117,119), residual
             slices as in temporal_ref.geometry
  loss       mpjpe (common/loss.py:11-17), run.py:478
  backward   torch autograd, run.py:485
  optimiser  optim.Adam(params, lr, amsgrad=True) (run.py:662), step run.py:487

The ops are torch-CPU functional ones (conv1d, batch_norm(training=True), relu,
autograd) — the kernels the reference's modules dispatch to — so with dropout 0 the
result equals the reference bit for bit (tests/test_oracle_golden.py, train_* goldens).
Dropout takes explicit keep masks (the reference draws them from torch's RNG, which a
device implementation cannot reproduce); the native trainer exports the masks it drew
(vp3d_train_dropout_mask) so the parity tests feed the same masks here.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from .temporal_ref import geometry


def _mask_cf(mask, B, L):
    """(B*L, C) channel-last keep mask -> (B, C, L) float tensor."""
    m = torch.as_tensor(np.asarray(mask)).reshape(B, L, -1).permute(0, 2, 1)
    return m.to(torch.float32)


def lifter_train_forward(params: Dict[str, torch.Tensor], x, filter_widths: Sequence[int], causal=False,
                         strided=False, dense=False, p: float = 0.0,
                         masks: Optional[List[np.ndarray]] = None, momentum: float = 0.1, eps: float = 1e-5,
                         relu_masks: Optional[List[np.ndarray]] = None):
    """Train-mode forward of TemporalModel (strided=False) / TemporalModelOptimized1f.

    params: state_dict-keyed tensors; the trainable ones may require grad, the BN
    running statistics are updated in place (F.batch_norm(training=True)).
    masks[l]: keep mask of conv layer l (0 = expand, then the block convs) as
    (B*L_l, C) uint8 rows, required when p > 0.
    relu_masks[l] (same layout, optional): take the ReLU decisions of another implementation
    (x * mask instead of relu(x)): an element whose BN output lies within rounding of 0 may
    fall on either side in two f32 implementations, and in a small batch one such element
    moves the BatchNorm gradients of its channel far more than rounding does."""
    xt = torch.as_tensor(np.asarray(x)) if not isinstance(x, torch.Tensor) else x
    B, T = xt.shape[0], xt.shape[1]
    pad, shift, convs = geometry(filter_widths, causal, strided, dense)
    w0 = filter_widths[0]

    def bn(h, name):
        return F.batch_norm(h, params[name + ".running_mean"], params[name + ".running_var"],
                            params[name + ".weight"], params[name + ".bias"], True, momentum, eps)

    def drop(h, layer):
        if p == 0:
            return h
        # at::native::dropout on CPU: noise = bernoulli(1 - p); noise.div_(1 - p); input * noise
        noise = _mask_cf(masks[layer], B, h.shape[2]).div_(1 - p)
        return h * noise

    def relu(h, layer):
        if relu_masks is None:
            return F.relu(h)
        return h * _mask_cf(relu_masks[layer], B, h.shape[2]).to(h.dtype)

    h = xt.reshape(B, T, -1).permute(0, 2, 1)
    h = drop(relu(bn(F.conv1d(h, params["expand_conv.weight"], None, stride=w0 if strided else 1),
                     "expand_bn"), 0), 0)
    for i, (k, d, s) in enumerate(convs):
        if strided:
            w = filter_widths[i + 1]
            res = h[:, :, shift[i + 1] + w // 2::w]
        else:
            pd, c = pad[i + 1], shift[i + 1]
            res = h[:, :, pd + c:h.shape[2] - pd + c]
        h = drop(relu(bn(F.conv1d(h, params[f"layers_conv.{2 * i}.weight"], None, stride=s, dilation=d),
                         f"layers_bn.{2 * i}"), 2 * i + 1), 2 * i + 1)
        h = res + drop(relu(bn(F.conv1d(h, params[f"layers_conv.{2 * i + 1}.weight"], None),
                               f"layers_bn.{2 * i + 1}"), 2 * i + 2), 2 * i + 2)
    h = F.conv1d(h, params["shrink.weight"], params["shrink.bias"])
    return h.permute(0, 2, 1).reshape(B, h.shape[2], -1, 3)


def mpjpe(pred, target):
    """common/loss.py:11-17."""
    assert pred.shape == target.shape
    return torch.mean(torch.norm(pred - target, dim=len(target.shape) - 1))


class TrainLoop:
    """The reference's iteration: forward, mpjpe, backward, Adam(amsgrad) step, on CPU."""

    def __init__(self, state: Dict[str, np.ndarray], filter_widths, causal=False, strided=False, dense=False,
                 lr=1e-3, amsgrad=True, momentum=0.1, eps=1e-5):
        self.params = {}
        for k, v in state.items():
            if k.endswith("num_batches_tracked"):
                continue
            t = torch.tensor(np.array(v, dtype=np.float32))
            if not (k.endswith("running_mean") or k.endswith("running_var")):
                t.requires_grad_(True)
            self.params[k] = t
        self.kw = dict(filter_widths=list(filter_widths), causal=causal, strided=strided, dense=dense)
        self.momentum, self.eps = momentum, eps
        self.opt = torch.optim.Adam([t for t in self.params.values() if t.requires_grad], lr=lr, amsgrad=amsgrad)

    def step(self, x, target, p=0.0, masks=None):
        """One iteration; returns (y, loss, grads) — the parameters are updated in place."""
        y = lifter_train_forward(self.params, x, p=p, masks=masks, momentum=self.momentum, eps=self.eps, **self.kw)
        loss = mpjpe(y, torch.as_tensor(np.asarray(target)))
        self.opt.zero_grad()
        loss.backward()
        grads = {k: t.grad.detach().clone() for k, t in self.params.items() if t.requires_grad}
        self.opt.step()
        return y.detach(), loss.detach(), grads

    def state(self) -> Dict[str, np.ndarray]:
        return {k: t.detach().numpy().copy() for k, t in self.params.items()}


def reference_epochs(state, fw, train_batches, test_sequences, n_epochs, lr=1e-3, lr_decay=0.95,
                     causal=False, total_epochs=None):
    """The epoch loop of run.py:451-558 on CPU: per epoch the training iterations over
    `train_batches()` (an iterable factory of (batch_cam, batch_3d, batch_2d) numpy
    batches), the evaluation of the eval-mode model on `test_sequences()` ((cam, 3d, 2d)
    per sequence), the lr decay and the BatchNorm momentum decay 0.1 -> 0.001
    (run.py:553-556).  Returns per-epoch (train, valid) losses in metres."""
    from .temporal_ref import lifter_forward
    total_epochs = total_epochs or n_epochs
    loop = TrainLoop(state, fw, causal=causal, lr=lr, amsgrad=True, momentum=0.1)
    out_train, out_valid = [], []
    for epoch in range(n_epochs):
        s = 0.0
        N = 0
        for bc, b3, b2 in train_batches():
            _, loss, _ = loop.step(b2.astype(np.float32), b3.astype(np.float32))
            n = b3.shape[0] * b3.shape[1]
            s += n * float(loss)
            N += n
        out_train.append(s / N)
        st = loop.state()
        s = 0.0
        N = 0
        with torch.no_grad():
            for bc, b3, b2 in test_sequences():
                y = lifter_forward(st, b2.astype(np.float32), fw, causal=causal)
                loss = mpjpe(y, torch.from_numpy(b3.astype(np.float32)))
                n = b3.shape[0] * b3.shape[1]
                s += n * float(loss)
                N += n
        out_valid.append(s / N)
        for g in loop.opt.param_groups:
            g["lr"] *= lr_decay
        e = epoch + 1
        loop.momentum = 0.1 * np.exp(-e / total_epochs * np.log(0.1 / 0.001))
    return out_train, out_valid
