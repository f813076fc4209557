"""Drop-in for the reference's ``common/models/CamLSTM.py``.

Same classes, constructor arguments, submodules and state_dict keys as
Bart-Weil/Dynamic-Camera-Augmented-VideoPose3D common/models/CamLSTM.py:

  CamLSTMBase     :11-44    ``sliding_window(inputs_2d, inputs_cam, window_size)``
  CoupledLSTM     :47-129   concat [2D | K.E] -> nn.LSTM (num_cells, zero state) -> last step
                            -> bn_lstm -> MLP head (Linear, BatchNorm1d, LeakyReLU, Dropout)*
  UncoupledLSTM   :132-257  raises NotImplementedError at construction, like the reference

Eval-mode ``forward`` / ``sliding_window`` on HIP tensors run libvp3d.so
(``vp3d_seq_forward`` / ``vp3d_seq_sliding_window``): the layer-0 input projection once per
frame on the f32 MFMA GEMM, the stacked recurrence in one persistent kernel per tile of 16
windows (csrc/seq_lifter.hip ``lstm_kernel``), the eval BatchNorms folded into the head's
GEMM epilogues.  CPU inputs and train mode raise.
"""
import torch.nn as nn

from vp3d_amd import _native as _N
from vp3d_amd.seq_lifter import NativeSeqLifter, NativeSeqModule

__all__ = ["CamLSTMBase", "CoupledLSTM", "UncoupledLSTM"]


class CamLSTMBase(NativeSeqModule, nn.Module):
    """Shared attributes and ``sliding_window`` (CamLSTM.py:11-44)."""

    cam_mat_shape = (3, 4)

    def __init__(self, num_joints_in, in_features, num_joints_out, out_features, hidden_size, num_cells,
                 head_layers, dropout=0.25):
        super().__init__()
        self.num_joints_in = num_joints_in
        self.in_features = in_features
        self.num_joints_out = num_joints_out
        self.out_features = out_features
        self.hidden_size = hidden_size
        self.num_cells = num_cells
        self.head_layers = head_layers
        self.dropout = dropout

    def sliding_window(self, inputs_2d, inputs_cam, window_size):
        _, T, J, _ = inputs_2d.shape
        if T - window_size + 1 <= 0:
            raise ValueError("window_size larger than sequence length")
        self._check_eval(inputs_2d)
        return self.native_lifter(inputs_2d.device).sliding_window(inputs_2d, inputs_cam, window_size)


class CoupledLSTM(CamLSTMBase):
    """Stacked-LSTM lifter over a window of [2D keypoints | camera matrix] frames (CamLSTM.py:47-129)."""

    def __init__(self, num_joints_in, in_features, num_joints_out, out_features, hidden_size, num_cells,
                 head_layers, dropout=0.25):
        super().__init__(num_joints_in, in_features, num_joints_out, out_features, hidden_size, num_cells,
                         head_layers, dropout)
        cin = num_joints_in * in_features + self.cam_mat_shape[0] * self.cam_mat_shape[1]
        self.lstm_layers = nn.LSTM(cin, hidden_size, num_cells, batch_first=True, dropout=dropout)
        self.bn_lstm = nn.BatchNorm1d(hidden_size)
        self.bn_layers = [self.bn_lstm]
        head = []
        width = hidden_size
        for h in head_layers:
            bn = nn.BatchNorm1d(h)
            self.bn_layers.append(bn)
            head += [nn.Linear(width, h), bn, nn.LeakyReLU(), nn.Dropout(dropout)]
            width = h
        head.append(nn.Linear(width, out_features * num_joints_out))
        self.mlp_layers = nn.Sequential(*head)

    def set_bn_momentum(self, momentum):
        for bn in self.bn_layers:
            bn.momentum = momentum

    def _make_native(self, state, device):
        return NativeSeqLifter(_N.SEQ_LSTM, self.num_joints_in, self.in_features, self.num_joints_out,
                               self.out_features, self.hidden_size, self.num_cells, self.head_layers, state, device,
                               eps=self.bn_lstm.eps)

    def forward(self, input_2d, input_cam):
        assert len(input_2d.shape) == 4 and len(input_cam.shape) == 4
        assert input_2d.shape[-2] == self.num_joints_in
        assert input_2d.shape[-1] == self.in_features
        assert input_cam.shape[-2] == self.cam_mat_shape[0]
        assert input_cam.shape[-1] == self.cam_mat_shape[1]
        self._check_eval(input_2d)
        return self.native_lifter(input_2d.device).forward(input_2d, input_cam)


class UncoupledLSTM(CamLSTMBase):
    """Not implemented on the reference's main branch either (CamLSTM.py:150)."""

    def __init__(self, *args, **kwargs):
        raise NotImplementedError("UncoupledLSTM data pipeline not implemented on main branch, "
                                  "use uncoupled-lstm branch instead")
