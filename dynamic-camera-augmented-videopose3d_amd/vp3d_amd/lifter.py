"""Python owner of a native lifter handle (vp3d_handle in include/vp3d.h).

`NativeLifter` is the thin object the drop-in `common.models.TemporalModel`
classes delegate their eval-mode forward to.  It owns one device copy of the
folded/packed weights and the activation workspace; it never computes anything
itself.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, List, Sequence

import numpy as np
import torch

from . import _native as N


def weight_order(n_widths: int) -> List[str]:
    """state_dict keys in the order vp3d_create expects (include/vp3d.h)."""
    keys = ["expand_conv.weight", "expand_bn.weight", "expand_bn.bias",
            "expand_bn.running_mean", "expand_bn.running_var"]
    for i in range(2 * (n_widths - 1)):
        keys += [f"layers_conv.{i}.weight", f"layers_bn.{i}.weight", f"layers_bn.{i}.bias",
                 f"layers_bn.{i}.running_mean", f"layers_bn.{i}.running_var"]
    keys += ["shrink.weight", "shrink.bias"]
    return keys


def _host_f32(v) -> np.ndarray:
    if isinstance(v, torch.Tensor):
        v = v.detach().to("cpu", torch.float32).contiguous().numpy()
    return np.ascontiguousarray(np.asarray(v, dtype=np.float32))


class NativeLifter:
    """One vp3d_handle on one HIP device."""

    def __init__(self, num_joints_in: int, in_features: int, num_joints_out: int,
                 filter_widths: Sequence[int], causal: bool, channels: int, dense: bool,
                 variant: int, state: dict, device=None, bn_eps: float = 1e-5):
        self._lib = N.load()
        self.n_widths = len(filter_widths)
        self.num_joints_out = num_joints_out
        self.cfg = N.make_cfg(num_joints_in, in_features, num_joints_out, filter_widths, causal,
                              channels, dense, variant, bn_eps)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None
                                   else torch.device(device).index or 0)
        self._h = ctypes.c_void_p()
        arrays, ptrs = self._pack(state)
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_create(ctypes.byref(self.cfg), ptrs, len(arrays),
                                          ctypes.byref(self._h)), "vp3d_create")
        self.n_layers = self._lib.vp3d_layer_count(self._h)

    def _pack(self, state: dict):
        keys = weight_order(self.n_widths)
        missing = [k for k in keys if k not in state]
        if missing:
            raise KeyError(f"missing state_dict keys: {missing}")
        arrays = [_host_f32(state[k]) for k in keys]
        ptrs = (ctypes.c_void_p * len(arrays))(*[a.ctypes.data for a in arrays])
        return arrays, ptrs

    def load_weights(self, state: dict) -> None:
        arrays, ptrs = self._pack(state)
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_load_weights(self._h, ptrs, len(arrays)), "vp3d_load_weights")

    # ---- shapes ----
    def receptive_field(self) -> int:
        return self._lib.vp3d_receptive_field(self._h)

    def total_causal_shift(self) -> int:
        return self._lib.vp3d_total_causal_shift(self._h)

    def out_frames(self, T: int) -> int:
        return self._lib.vp3d_out_frames(self._h, int(T))

    # ---- compute ----
    def reserve(self, B: int, T: int, dtype: str = "fp32") -> None:
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_reserve(self._h, int(B), int(T), N.DTYPES[dtype]), "vp3d_reserve")

    def forward(self, x: torch.Tensor, dtype: str = "fp32", out: torch.Tensor | None = None
                ) -> torch.Tensor:
        """x: (B, T, J_in, F) float32 on this handle's device -> (B, T', J_out, 3) float32."""
        if x.device != self.device:
            raise RuntimeError(f"input on {x.device}, model on {self.device}")
        if x.dtype != torch.float32:
            x = x.float()
        x = x.contiguous()
        B, T = int(x.shape[0]), int(x.shape[1])
        T_out = self.out_frames(T)
        if T_out < 1:
            raise RuntimeError(f"input of {T} frames is invalid for receptive field "
                               f"{self.receptive_field()}")
        if out is None:
            out = torch.empty((B, T_out, self.num_joints_out, 3), dtype=torch.float32,
                              device=self.device)
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_forward(self._h, x.data_ptr(), B, T, out.data_ptr(),
                                           N.DTYPES[dtype], N.stream_ptr(self.device)),
                    "vp3d_forward")
        return out

    def forward_windows(self, seqs, pairs: torch.Tensor, window: int, lead: int,
                        concat_cams: bool = False, dtype: str = "fp32",
                        out: torch.Tensor | None = None) -> torch.Tensor:
        """Forward of windows gathered on the fly from `seqs` (a pipeline.DeviceSequences):
        window b = frames [start_b - lead, start_b - lead + window) of sequence seq_b,
        edge-clamped; with concat_cams the 12 K.E channels follow each frame's keypoints
        (vp3d_forward_windows: ChunkedGenerator batch + camera concat + TemporalModel forward,
        the gather fused into the expand conv on the 16-bit path)."""
        def _idx(d):
            d = torch.device(d)
            return (d.type, d.index if d.index is not None else torch.cuda.current_device())
        if _idx(pairs.device) != _idx(self.device) or _idx(seqs.kps.device) != _idx(self.device):
            raise RuntimeError("pairs / sequences must live on the model's device")
        pairs = pairs.contiguous().to(torch.int32)
        B = int(pairs.shape[0])
        T_out = self.out_frames(window)
        if T_out < 1:
            raise RuntimeError(f"window of {window} frames is invalid for receptive field "
                               f"{self.receptive_field()}")
        cams = None
        if concat_cams:
            if seqs.cam is None:
                raise ValueError("no cameras loaded")
            cams = seqs.cam.data_ptr()
        if out is None:
            out = torch.empty((B, T_out, self.num_joints_out, 3), dtype=torch.float32,
                              device=self.device)
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_forward_windows(
                self._h, seqs.kps.data_ptr(), seqs.f2, cams, seqs.seq_off.data_ptr(),
                seqs.seq_len.data_ptr(), pairs.data_ptr(), B, int(window), int(lead), out.data_ptr(),
                N.DTYPES[dtype], N.stream_ptr(self.device)), "vp3d_forward_windows")
        return out

    def sync_status(self) -> None:
        """Synchronise the current stream; raise RuntimeError once if a launch of this lifter
        reported a device-side fault, and clear it (vp3d_sync_status).  The fault kinds:
          * split-K timeout -- an owner tile of a split partial round stopped waiting for its
            helper units (its outputs are wrong); refuses EVERY forward until cleared here;
          * f16x3 range / non-finite -- an activation split into f16 halves was past |x| <=
            65,504, or the poses came out non-finite; refuses f16x3 forwards only (run those
            inputs in fp32).
        A forward raises a pending fault of an earlier forward at entry; the last forward of
        a run is only checked by calling this (vp3d_amd.evaluate does, after its loop)."""
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_sync_status(self._h, N.stream_ptr(self.device)), "vp3d_sync_status")

    # ---- profiling ----
    def profile(self, enable: bool) -> None:
        N.check(self._lib.vp3d_profile_enable(self._h, 1 if enable else 0))

    def profile_layers(self, layers=None) -> None:
        """Time only `layers` (indices; None = all) while profiling is enabled."""
        mask = (1 << 64) - 1 if layers is None else sum(1 << int(i) for i in layers)
        N.check(self._lib.vp3d_profile_layers(self._h, mask))

    def profile_reset(self) -> None:
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_profile_reset(self._h))

    def profile_read(self):
        n = self.n_layers
        ms = (ctypes.c_double * n)()
        cnt = (ctypes.c_int64 * n)()
        fl = (ctypes.c_double * n)()
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_profile_read(self._h, ctypes.addressof(ms),
                                                ctypes.addressof(cnt), ctypes.addressof(fl)))
        return [dict(layer=i, ms_total=ms[i], launches=cnt[i], flop=fl[i]) for i in range(n)]

    def close(self) -> None:
        if self._h:
            self._lib.vp3d_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
