"""ORACLE (test infrastructure only): CPU restatement of the lifter forward.

Follows reference common/models/TemporalModel.py:
  forward            :62-76   (B,T,J,F) -> view (B,T,J*F) -> permute -> blocks -> (B,T',J_out,3)
  dilated blocks     :126-138 res = x[:, :, pad+shift : L-pad+shift]; relu(bn(conv_dil)); 1x1; add
  strided blocks     :188-198 res = x[:, :, shift + w//2 :: w];        relu(bn(conv_s));  1x1; add
  geometry           :31, :107-111, :173-177 (pad / causal_shift / dilation)

The op sequence is torch-CPU functional (conv1d -> batch_norm(eval) -> relu),
i.e. the very kernels the reference's nn.Modules dispatch to, so with the same
weights the result is bit-identical to the reference in fp32.  ``dtype=float64``
gives an exact-arithmetic yardstick for tolerance statements.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def geometry(filter_widths, causal, strided, dense=False):
    """(pad, causal_shift, [(kernel, dilation, stride)] per block) as the reference builds them."""
    pad = [filter_widths[0] // 2]
    shift = [filter_widths[0] // 2 if causal else 0]
    convs = []
    dil = filter_widths[0]
    for w in filter_widths[1:]:
        pad.append((w - 1) * dil // 2)
        if strided:
            shift.append(w // 2 if causal else 0)
            convs.append((w, 1, w))
        else:
            shift.append((w // 2) * dil if causal else 0)
            convs.append((2 * pad[-1] + 1, 1, 1) if dense else (w, dil, 1))
        dil *= w
    return pad, shift, convs


def receptive_field(filter_widths):
    pad, _, _ = geometry(filter_widths, False, False)
    return 1 + 2 * sum(pad)


def _t(v, dtype):
    if isinstance(v, torch.Tensor):
        return v.detach().to("cpu", dtype)
    return torch.from_numpy(np.asarray(v)).to(dtype)


def lifter_forward(state, x, filter_widths, causal=False, strided=False, dense=False,
                   dtype=torch.float32, eps=1e-5, num_threads=None):
    """Eval-mode forward of TemporalModel (strided=False) / TemporalModelOptimized1f
    (strided=True) with the given state_dict.  x: (B, T, J, F) array or tensor.
    Returns a float tensor (B, T', J_out, 3) in `dtype`."""
    if num_threads is not None:
        torch.set_num_threads(num_threads)
    sd = {k: _t(v, dtype) for k, v in state.items() if not k.endswith("num_batches_tracked")}
    xt = _t(x, dtype)
    B, T = xt.shape[0], xt.shape[1]
    pad, shift, convs = geometry(filter_widths, causal, strided, dense)
    w0 = filter_widths[0]

    def bn(h, name):
        return F.batch_norm(h, sd[name + ".running_mean"], sd[name + ".running_var"],
                            sd[name + ".weight"], sd[name + ".bias"], False, 0.1, eps)

    with torch.no_grad():
        h = xt.reshape(B, T, -1).permute(0, 2, 1)
        h = F.conv1d(h, sd["expand_conv.weight"], None, stride=w0 if strided else 1)
        h = F.relu(bn(h, "expand_bn"))
        for i, (k, d, s) in enumerate(convs):
            if strided:
                w = filter_widths[i + 1]
                res = h[:, :, shift[i + 1] + w // 2::w]
            else:
                p, c = pad[i + 1], shift[i + 1]
                res = h[:, :, p + c:h.shape[2] - p + c]
            h = F.relu(bn(F.conv1d(h, sd[f"layers_conv.{2 * i}.weight"], None, stride=s, dilation=d),
                          f"layers_bn.{2 * i}"))
            h = res + F.relu(bn(F.conv1d(h, sd[f"layers_conv.{2 * i + 1}.weight"], None),
                                f"layers_bn.{2 * i + 1}"))
        h = F.conv1d(h, sd["shrink.weight"], sd["shrink.bias"])
        return h.permute(0, 2, 1).reshape(B, h.shape[2], -1, 3)


def conv_flops_per_pose(filter_widths, cin, channels, jout, strided):
    """Algorithmic FLOP (2 x conv MACs, BN/ReLU/add excluded) for one output pose:
    Optimized1f on one RF window, or the asymptotic per-frame cost of the dilated model."""
    pad, shift, convs = geometry(filter_widths, False, strided)
    w0 = filter_widths[0]
    if strided:
        L = receptive_field(filter_widths)
        L = (L - w0) // w0 + 1
        macs = L * channels * cin * w0
        for (k, d, s) in convs:
            L = (L - k) // s + 1
            macs += L * channels * channels * k + L * channels * channels
        macs += L * jout * 3 * channels
        return 2 * macs
    macs = channels * cin * w0
    for (k, d, s) in convs:
        macs += channels * channels * k + channels * channels
    macs += jout * 3 * channels
    return 2 * macs
