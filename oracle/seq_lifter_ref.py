"""ORACLE (test infrastructure only): CPU restatement of the fork's trajectory-conditioned
lifters in eval mode.

Follows reference common/models/CamTransformer.py and CamLSTM.py:
  PositionalEncoding          CamTransformer.py:5-34   x + pe[:, :T]  (dropout: identity in eval)
  CoupledTransformer.forward  CamTransformer.py:165-205 concat(flat 2D, flat K.E) -> input_projection
                              -> + pe -> pre_transformer_norm -> nn.TransformerEncoder (post-norm
                              layers: x = norm1(x + sa(x)); x = norm2(x + linear2(relu(linear1(x)))))
                              -> last time step -> MLP head (Linear, LeakyReLU, Dropout)*
  CoupledLSTM.forward         CamLSTM.py:104-129 concat -> nn.LSTM (2 cells, zero state) -> last step
                              -> bn_lstm -> MLP head (Linear, BatchNorm1d, LeakyReLU, Dropout)*
  sliding_window              CamTransformer.py:72-92 / CamLSTM.py:33-44: windows of `window_size`
                              frames at stride 1 over one (padded) sequence, one output per window

torch-CPU functional ops (F.linear, F.layer_norm, softmax attention, explicit LSTM cell);
pinned to the reference's own outputs by tests/test_oracle_seq_lifter.py (golden fixtures
cam_transformer.npz / cam_lstm.npz made by tests/golden/make_golden.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F


def _t(v, dtype=torch.float32):
    return v.detach().to(dtype) if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v)).to(dtype)


def positional_encoding(d_model: int, max_len: int = 5000) -> torch.Tensor:
    """The sinusoid table of PositionalEncoding.__init__ (CamTransformer.py:17-24)."""
    pe = torch.zeros(max_len, d_model)
    position = torch.arange(0, max_len, dtype=torch.float).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, d_model, 2).float() * (-math.log(10000.0) / d_model))
    pe[:, 0::2] = torch.sin(position * div_term)
    pe[:, 1::2] = torch.cos(position * div_term)
    return pe


def _concat(x2d, xcam, dtype):
    x2d, xcam = _t(x2d, dtype), _t(xcam, dtype)
    B, T = x2d.shape[0], x2d.shape[1]
    return torch.cat([x2d.reshape(B, T, -1), xcam.reshape(B, T, -1)], dim=2)


def _mlp_head(sd, h, prefix, n_linear, bn=False, eps=1e-5):
    """Linear [-> BatchNorm1d] -> LeakyReLU (-> Dropout) ... -> Linear (eval)."""
    idx = 0
    for i in range(n_linear):
        h = F.linear(h, sd[f"{prefix}.{idx}.weight"], sd[f"{prefix}.{idx}.bias"])
        idx += 1
        if i == n_linear - 1:
            break
        if bn:
            h = F.batch_norm(h, sd[f"{prefix}.{idx}.running_mean"], sd[f"{prefix}.{idx}.running_var"],
                             sd[f"{prefix}.{idx}.weight"], sd[f"{prefix}.{idx}.bias"], False, 0.1, eps)
            idx += 1
        h = F.leaky_relu(h, 0.01)
        idx += 2  # LeakyReLU, Dropout
    return h


def transformer_forward(state, x2d, xcam, n_heads: int, num_layers: int, n_head_layers: int,
                        dtype=torch.float32, eps: float = 1e-5):
    """CoupledTransformer.forward in eval mode: (B, T, J, 2), (B, T, 3, 4) -> (B, 1, J_out, 3)."""
    sd = {k: _t(v, dtype) for k, v in state.items() if not k.endswith("num_batches_tracked")}
    x = _concat(x2d, xcam, dtype)
    B, T, _ = x.shape
    d = sd["input_projection.weight"].shape[0]
    pe = sd.get("positional_encoding.pe")
    pe = positional_encoding(d).to(dtype) if pe is None else pe.reshape(-1, d)
    h = F.linear(x, sd["input_projection.weight"], sd["input_projection.bias"]) + pe[:T]
    h = F.layer_norm(h, (d,), sd["pre_transformer_norm.weight"], sd["pre_transformer_norm.bias"], eps)
    dh = d // n_heads
    for li in range(num_layers):
        p = f"transformer_encoder.layers.{li}."
        qkv = F.linear(h, sd[p + "self_attn.in_proj_weight"], sd[p + "self_attn.in_proj_bias"])
        q, k, v = qkv.split(d, dim=2)
        q = q.reshape(B, T, n_heads, dh).transpose(1, 2)
        k = k.reshape(B, T, n_heads, dh).transpose(1, 2)
        v = v.reshape(B, T, n_heads, dh).transpose(1, 2)
        att = torch.softmax((q @ k.transpose(-1, -2)) / math.sqrt(dh), dim=-1)
        o = (att @ v).transpose(1, 2).reshape(B, T, d)
        sa = F.linear(o, sd[p + "self_attn.out_proj.weight"], sd[p + "self_attn.out_proj.bias"])
        h = F.layer_norm(h + sa, (d,), sd[p + "norm1.weight"], sd[p + "norm1.bias"], eps)
        ff = F.linear(F.relu(F.linear(h, sd[p + "linear1.weight"], sd[p + "linear1.bias"])),
                      sd[p + "linear2.weight"], sd[p + "linear2.bias"])
        h = F.layer_norm(h + ff, (d,), sd[p + "norm2.weight"], sd[p + "norm2.bias"], eps)
    out = _mlp_head(sd, h[:, -1, :], "mlp_layers", n_head_layers + 1)
    return out.reshape(B, 1, -1, 3)


def lstm_forward(state, x2d, xcam, hidden: int, num_cells: int, n_head_layers: int,
                 dtype=torch.float32, eps: float = 1e-5):
    """CoupledLSTM.forward in eval mode (nn.LSTM gate order i, f, g, o; zero initial state)."""
    sd = {k: _t(v, dtype) for k, v in state.items() if not k.endswith("num_batches_tracked")}
    x = _concat(x2d, xcam, dtype)
    B, T, _ = x.shape
    seq = x
    for l in range(num_cells):
        wi, wh = sd[f"lstm_layers.weight_ih_l{l}"], sd[f"lstm_layers.weight_hh_l{l}"]
        bi, bh = sd[f"lstm_layers.bias_ih_l{l}"], sd[f"lstm_layers.bias_hh_l{l}"]
        gx = F.linear(seq, wi, bi)
        h = torch.zeros(B, hidden, dtype=dtype)
        c = torch.zeros(B, hidden, dtype=dtype)
        outs = []
        for t in range(T):
            g = gx[:, t] + F.linear(h, wh, bh)
            i, f, gg, o = g.split(hidden, dim=1)
            c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
            h = torch.sigmoid(o) * torch.tanh(c)
            outs.append(h)
        seq = torch.stack(outs, dim=1)
    last = F.batch_norm(seq[:, -1, :], sd["bn_lstm.running_mean"], sd["bn_lstm.running_var"],
                        sd["bn_lstm.weight"], sd["bn_lstm.bias"], False, 0.1, eps)
    out = _mlp_head(sd, last, "mlp_layers", n_head_layers + 1, bn=True)
    return out.reshape(B, 1, -1, 3)


def sliding_windows(x2d, xcam, window: int):
    """The unfold of sliding_window (CamTransformer.py:86-89): (1, L, ...) -> (L - window + 1, window, ...)."""
    x2d, xcam = _t(x2d), _t(xcam)
    n = x2d.shape[1] - window + 1
    idx = torch.arange(n)[:, None] + torch.arange(window)[None, :]
    return x2d[0][idx], xcam[0][idx]
