"""Drop-in for the reference's ``common/models/CamTransformer.py``.

Same classes, constructor arguments, submodules and state_dict keys as
Bart-Weil/Dynamic-Camera-Augmented-VideoPose3D common/models/CamTransformer.py:

  PositionalEncoding   :5-34     sinusoid table buffer ``pe`` (1, max_len, d_model)
  CamTransformerBase   :37-92    ``sliding_window(inputs_2d, inputs_cam, window_size)``
  CoupledTransformer   :95-205   concat [2D | K.E] -> input_projection -> + pe ->
                                 pre_transformer_norm -> TransformerEncoder (post-norm, ReLU)
                                 -> last step -> MLP head (Linear, LeakyReLU, Dropout)*

The nn modules only hold the parameters.  Eval-mode ``forward`` and ``sliding_window`` on
HIP tensors run libvp3d.so (``vp3d_seq_forward`` / ``vp3d_seq_sliding_window``): every Linear
on the f32 MFMA GEMM, LayerNorm and attention kernels of csrc/seq_lifter.hip; the
last encoder layer evaluates only the last query (the only output the model keeps), and
sliding windows share one input projection per frame.  CPU inputs and train mode raise.
"""
import math

import torch
import torch.nn as nn

from vp3d_amd import _native as _N
from vp3d_amd.seq_lifter import NativeSeqLifter, NativeSeqModule

__all__ = ["PositionalEncoding", "CamTransformerBase", "CoupledTransformer"]


class PositionalEncoding(nn.Module):
    """Adds the sinusoidal position table (CamTransformer.py:5-34); dropout after it."""

    def __init__(self, d_model: int, dropout: float = 0.1, max_len: int = 5000):
        super().__init__()
        self.dropout = nn.Dropout(p=dropout)
        pos = torch.arange(max_len, dtype=torch.float).unsqueeze(1)
        freq = torch.exp(torch.arange(0, d_model, 2).float() * (-math.log(10000.0) / d_model))
        table = torch.zeros(max_len, d_model)
        table[:, 0::2] = torch.sin(pos * freq)
        table[:, 1::2] = torch.cos(pos * freq)
        self.register_buffer("pe", table.unsqueeze(0))

    def forward(self, x):
        return self.dropout(x + self.pe[:, :x.size(1)])


class CamTransformerBase(NativeSeqModule, nn.Module):
    """Shared attributes and ``sliding_window`` (CamTransformer.py:37-92)."""

    cam_mat_shape = (3, 4)

    def __init__(self, num_joints_in, in_features, num_joints_out, out_features, d_model, num_layers, n_heads,
                 dim_feedforward, head_layers, dropout=0.25):
        super().__init__()
        self.num_joints_in = num_joints_in
        self.in_features = in_features
        self.num_joints_out = num_joints_out
        self.out_features = out_features
        self.d_model = d_model
        self.num_layers = num_layers
        self.n_heads = n_heads
        self.dim_feedforward = dim_feedforward
        self.head_layers = head_layers
        self.dropout = dropout

    def sliding_window(self, inputs_2d, inputs_cam, window_size):
        """One prediction per window of `window_size` frames at stride 1 over the single
        (padded) sequence inputs_2d (1, T, J, F) / inputs_cam (1, T, 3, 4) ->
        (1, T - window_size + 1, J_out, out_features)."""
        _, T, J, _ = inputs_2d.shape
        if T - window_size + 1 <= 0:
            raise ValueError("window_size larger than sequence length")
        self._check_eval(inputs_2d)
        return self.native_lifter(inputs_2d.device).sliding_window(inputs_2d, inputs_cam, window_size)


class CoupledTransformer(CamTransformerBase):
    """Transformer lifter over a window of [2D keypoints | camera matrix] frames
    (CamTransformer.py:95-205)."""

    def __init__(self, num_joints_in, in_features, num_joints_out, out_features, d_model, num_layers, n_heads,
                 dim_feedforward, head_layers, dropout=0.25):
        super().__init__(num_joints_in, in_features, num_joints_out, out_features, d_model, num_layers, n_heads,
                         dim_feedforward, head_layers, dropout)
        concat_dim = num_joints_in * in_features + self.cam_mat_shape[0] * self.cam_mat_shape[1]
        self.input_projection = nn.Linear(concat_dim, d_model)
        self.positional_encoding = PositionalEncoding(d_model, dropout)
        self.pre_transformer_norm = nn.LayerNorm(d_model)
        layer = nn.TransformerEncoderLayer(d_model=d_model, nhead=n_heads, dim_feedforward=dim_feedforward,
                                           dropout=dropout, batch_first=True)
        self.transformer_encoder = nn.TransformerEncoder(layer, num_layers=num_layers, enable_nested_tensor=False)
        head = []
        width = d_model
        for h in head_layers:
            head += [nn.Linear(width, h), nn.LeakyReLU(), nn.Dropout(dropout)]
            width = h
        head.append(nn.Linear(width, out_features * num_joints_out))
        self.mlp_layers = nn.Sequential(*head)

    def _make_native(self, state, device):
        return NativeSeqLifter(_N.SEQ_TRANSFORMER, self.num_joints_in, self.in_features, self.num_joints_out,
                               self.out_features, self.d_model, self.num_layers, self.head_layers, state, device,
                               n_heads=self.n_heads, dim_feedforward=self.dim_feedforward,
                               max_len=int(self.positional_encoding.pe.shape[1]),
                               eps=self.pre_transformer_norm.eps)

    def forward(self, input_2d, input_cam):
        """(B, T, J_in, F), (B, T, 3, 4) -> (B, 1, J_out, out_features)."""
        assert len(input_2d.shape) == 4 and len(input_cam.shape) == 4, "Invalid input dims"
        assert input_2d.shape[-2] == self.num_joints_in and input_2d.shape[-1] == self.in_features, \
            "Unexpected 2D input shape"
        assert input_cam.shape[-2] == self.cam_mat_shape[0] and input_cam.shape[-1] == self.cam_mat_shape[1], \
            "Unexpected camera matrix shape"
        self._check_eval(input_2d)
        return self.native_lifter(input_2d.device).forward(input_2d, input_cam)
