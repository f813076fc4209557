"""Python owner of a native trajectory-lifter handle (vp3d_seq_lifter, include/vp3d.h).

The drop-in `common.models.CamTransformer` / `common.models.CamLSTM` modules delegate their
eval-mode `forward` and `sliding_window` to it.  It holds one
device copy of the packed weights; it computes nothing itself.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np
import torch

from . import _native as N


def _host_f32(v) -> np.ndarray:
    if isinstance(v, torch.Tensor):
        v = v.detach().to("cpu", torch.float32).contiguous().numpy()
    return np.ascontiguousarray(np.asarray(v, dtype=np.float32))


class NativeSeqLifter:
    def __init__(self, kind: int, num_joints_in: int, in_features: int, num_joints_out: int, out_features: int,
                 d_model: int, num_layers: int, head_layers: Sequence[int], state: dict, device,
                 n_heads: int = 1, dim_feedforward: int = 0, max_len: int = 0, eps: float = 1e-5):
        self._lib = N.load()
        cfg = N.vp3d_seq_cfg()
        cfg.kind = kind
        cfg.num_joints_in, cfg.in_features = num_joints_in, in_features
        cfg.num_joints_out, cfg.out_features = num_joints_out, out_features
        cfg.d_model, cfg.num_layers = d_model, num_layers
        cfg.n_heads, cfg.dim_feedforward = n_heads, dim_feedforward
        if not 1 <= len(head_layers) <= N.SEQ_MAX_HEAD:
            raise AssertionError(f"1..{N.SEQ_MAX_HEAD} head layers are supported")
        cfg.n_head_layers = len(head_layers)
        for i, v in enumerate(head_layers):
            cfg.head_layers[i] = int(v)
        cfg.max_len, cfg.eps = max_len, eps
        self.cfg = cfg
        self.num_joints_out, self.out_features = num_joints_out, out_features
        self.device = torch.device(device)
        arrays = [_host_f32(v) for k, v in state.items() if not k.endswith("num_batches_tracked")]
        n = self._lib.vp3d_seq_weight_count(ctypes.byref(cfg))
        if n != len(arrays):
            raise RuntimeError(f"vp3d: {len(arrays)} state tensors for a configuration expecting {n}")
        ptrs = (ctypes.c_void_p * len(arrays))(*[a.ctypes.data for a in arrays])
        self._h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_seq_create(ctypes.byref(cfg), ptrs, len(arrays), ctypes.byref(self._h)),
                    "vp3d_seq_create")

    def _prep(self, t):
        if t.device != self.device:
            raise RuntimeError(f"input on {t.device}, model on {self.device}")
        return t.contiguous().float()

    def forward(self, input_2d: torch.Tensor, input_cam: torch.Tensor) -> torch.Tensor:
        x2, xc = self._prep(input_2d), self._prep(input_cam)
        B, T = int(x2.shape[0]), int(x2.shape[1])
        y = torch.empty((B, 1, self.num_joints_out, self.out_features), device=self.device)
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_seq_forward(self._h, x2.data_ptr(), xc.data_ptr(), B, T, y.data_ptr(),
                                               N.stream_ptr(self.device)), "vp3d_seq_forward")
        return y

    def sliding_window(self, input_2d: torch.Tensor, input_cam: torch.Tensor, window: int) -> torch.Tensor:
        """input_2d (1, L, J, F), input_cam (1, L, 3, 4) -> (1, L - window + 1, J_out, out_features)."""
        x2, xc = self._prep(input_2d), self._prep(input_cam)
        L = int(x2.shape[1])
        n = L - int(window) + 1
        if n <= 0:
            raise ValueError("window_size larger than sequence length")
        y = torch.empty((1, n, self.num_joints_out, self.out_features), device=self.device)
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_seq_sliding_window(self._h, x2.data_ptr(), xc.data_ptr(), L, int(window),
                                                      y.data_ptr(), N.stream_ptr(self.device)),
                    "vp3d_seq_sliding_window")
        return y

    def close(self):
        if self._h:
            self._lib.vp3d_seq_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class NativeSeqModule:
    """Mixin for the drop-in sequence-lifter modules: a NativeSeqLifter per device, re-packed
    whenever a parameter or buffer was replaced or modified in place."""

    def _native_key(self, device):
        return (str(device),) + tuple((t.data_ptr(), t._version) for t in self.state_dict(keep_vars=True).values())

    def native_lifter(self, device) -> NativeSeqLifter:
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("vp3d: the sequence lifters run on the MI355X kernels only (no CPU fallback)")
        key = self._native_key(device)
        cached = getattr(self, "_native", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        lifter = self._make_native(dict(self.state_dict()), device)
        self._native = (key, lifter)
        return lifter

    def _check_eval(self, x):
        if not x.is_cuda:
            raise RuntimeError("vp3d: the sequence lifters run on the MI355X kernels only (no CPU fallback); "
                               "call model.cuda() and pass CUDA tensors")
        if self.training:
            raise NotImplementedError("vp3d: training the trajectory lifters is not on the MI355X path "
                                      "(eval-mode forward and sliding_window are); call model.eval()")
