"""Causal streaming inference (BASELINE config 5): one 2D frame in, one 3D pose out.

Wraps vp3d_stream (include/vp3d.h): a batch of steps is one layer-pipelined persistent
launch (csrc/stream_pipe.hip: every CU owns one layer's channel slice with its weights
resident in VGPRs as f32 -- exact fp32 weights for dtype "fp32", 16-bit weights widened
for "fp16" / "bf16" -- and layer outputs are handed between CUs in-launch); shapes the
pipeline does not cover fall back to stream_persist.hip (16-bit weights in LDS) or to one
GEMV launch per layer (csrc/stream_step.hip).  For a causal dilated TemporalModel
(reference TemporalModel.py:79-138 with causal=True), pose k of the stream equals
frame k of the reference's whole-sequence evaluation of the edge-padded
sequence (UnchunkedGenerator, generators.py:193-198, causal_shift = pad).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native as N


class CausalStream:
    def __init__(self, lifter, dtype: str = "fp16"):
        """lifter: a NativeLifter (``model.native_lifter()``) of a causal TemporalModel."""
        self._lib = N.load()
        self.lifter = lifter
        self.device = lifter.device
        self.dtype = dtype
        self._s = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_stream_create(lifter._h, N.DTYPES[dtype], ctypes.byref(self._s)),
                    "vp3d_stream_create")
        fin, fout, q = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int()
        N.check(self._lib.vp3d_stream_io(self._s, ctypes.byref(fin), ctypes.byref(fout), ctypes.byref(q)))
        self._in_ptr, self._out_ptr, self.queue_len = fin.value, fout.value, q.value
        self.n_in = lifter.cfg.num_joints_in * lifter.cfg.in_features
        self.n_out = lifter.cfg.num_joints_out * 3
        self._graph_stream = None

    def reset(self) -> None:
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_stream_reset(self._s, N.stream_ptr(self.device)))

    def step(self, frame: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """frame: (J_in, F) float32 on the device -> (J_out, 3) float32."""
        if not frame.is_cuda:
            raise RuntimeError("vp3d: stream frames must be HIP device tensors (no CPU fallback)")
        frame = frame.contiguous().float()
        assert frame.numel() == self.n_in
        if out is None:
            out = torch.empty((self.n_out // 3, 3), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_stream_step(self._s, frame.data_ptr(), out.data_ptr(),
                                               N.stream_ptr(self.device)), "vp3d_stream_step")
        return out

    def frames_seen(self) -> int:
        return int(self._lib.vp3d_stream_frames_seen(self._s))

    @property
    def persistent(self) -> bool:
        """True when steps run as one persistent launch per batch (weights resident on
        chip: mode 'pipe' or 'persist'); False for one GEMV launch per layer
        (VP3D_STREAM_MODE=launches, or a shape neither persistent form covers)."""
        return bool(self._lib.vp3d_stream_persistent(self._s))

    @property
    def mode(self) -> str:
        """'pipe' (layer-pipelined persistent launch, stream_pipe.hip), 'persist' (every CU
        runs every layer, weights in LDS, stream_persist.hip) or 'launches' (GEMV per layer)."""
        return {2: "pipe", 1: "persist", 0: "launches"}[int(self._lib.vp3d_stream_mode(self._s))]

    def check(self) -> None:
        """Synchronise and raise if a persistent launch gave up waiting on another CU."""
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_stream_status(self._s), "vp3d_stream_status")

    # ---- serving: the pipelined launch stays resident, frames posted from the host ----
    def serve(self, idle_ms: float = 200.0, stream: torch.cuda.Stream | None = None) -> "Serving":
        """Context manager for real-time use, one frame in flight (config 5's single-frame
        latency): the layer-pipelined launch (mode 'pipe') stays resident with its weights
        in VGPRs; `post(frame)` writes a host frame into pinned memory, `wait(t)` spins on
        pinned memory until pose t is there -- no launch, copy or graph per frame.  The
        launch ends itself after `idle_ms` without a frame."""
        return Serving(self, idle_ms, stream)

    def trace(self):
        """Per-frame device clocks of the layer-pipelined launch (VP3D_STREAM_TRACE=n set
        before the stream was created): returns (clocks, role_first_wg) with clocks of shape
        (workgroups, n, 11) -- [..., 0] input complete, [..., 1 + w] wave w's first output
        stored, 100 MHz ticks, 0 = not recorded; [..., 9], [..., 10] the shader clock counter
        at [..., 0] and [..., 1] -- for the first n frames of the last launch, then clears them."""
        roles, frames = ctypes.c_int32(), ctypes.c_int32()
        N.check(self._lib.vp3d_stream_trace(self._s, None, 0, None, ctypes.byref(roles), ctypes.byref(frames)),
                "vp3d_stream_trace")
        first = np.zeros(roles.value + 1, np.int32)
        N.check(self._lib.vp3d_stream_trace(self._s, None, 0, first.ctypes.data, ctypes.byref(roles),
                                            ctypes.byref(frames)), "vp3d_stream_trace")
        out = np.zeros((int(first[-1]), frames.value, 11), np.uint64)
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_stream_trace(self._s, out.ctypes.data, out.size, first.ctypes.data,
                                                ctypes.byref(roles), ctypes.byref(frames)), "vp3d_stream_trace")
        return out, first

    # ---- hipGraph replay: steps read the device frame queue, write the pose ring ----
    def io_tensors(self):
        """(frame_queue (Q, J_in*F), pose_ring (Q, J_out*3)) views of the device buffers:
        step t reads frame slot t % Q and writes pose slot t % Q."""
        Q = self.queue_len
        fin = _wrap(self._in_ptr, Q * self.n_in, self.device).view(Q, self.n_in)
        fout = _wrap(self._out_ptr, Q * self.n_out, self.device).view(Q, self.n_out)
        return fin, fout

    def capture(self, stream: torch.cuda.Stream, steps: int = 1) -> None:
        """Capture `steps` consecutive steps into one hipGraph."""
        self._graph_stream = stream
        with torch.cuda.device(self.device):
            N.check(self._lib.vp3d_stream_graph_capture(self._s, stream.cuda_stream, int(steps)),
                    "vp3d_stream_graph_capture")

    def replay(self, stream: torch.cuda.Stream | None = None) -> None:
        s = stream if stream is not None else self._graph_stream
        N.check(self._lib.vp3d_stream_graph_launch(self._s, s.cuda_stream), "vp3d_stream_graph_launch")

    def close(self) -> None:
        if self._s:
            self._lib.vp3d_stream_destroy(self._s)
            self._s = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Serving:
    """A resident serve launch of a CausalStream (vp3d_stream_serve_*)."""

    def __init__(self, st: CausalStream, idle_ms: float, stream):
        self.st, self.idle_ms = st, float(idle_ms)
        self.stream = stream if stream is not None else torch.cuda.Stream(st.device)
        self._pose = np.empty(st.n_out, dtype=np.float32)

    def __enter__(self):
        with torch.cuda.device(self.st.device):
            N.check(self.st._lib.vp3d_stream_serve_begin(self.st._s, self.stream.cuda_stream, self.idle_ms),
                    "vp3d_stream_serve_begin")
        return self

    def post(self, frame) -> int:
        """Post one frame ((J_in, F) host float32); returns its stream index."""
        f = np.ascontiguousarray(np.asarray(frame, dtype=np.float32)).reshape(-1)
        assert f.size == self.st.n_in
        t = ctypes.c_int64()
        N.check(self.st._lib.vp3d_stream_serve_post(self.st._s, f.ctypes.data, ctypes.byref(t)),
                "vp3d_stream_serve_post")
        return int(t.value)

    def wait(self, t: int, timeout_ms: float = 1000.0) -> np.ndarray:
        """Pose (J_out, 3) of frame t (host float32)."""
        out = np.empty(self.st.n_out, dtype=np.float32)
        N.check(self.st._lib.vp3d_stream_serve_wait(self.st._s, int(t), out.ctypes.data, float(timeout_ms)),
                "vp3d_stream_serve_wait")
        return out.reshape(-1, 3)

    def step(self, frame, timeout_ms: float = 1000.0) -> np.ndarray:
        """post + wait in one library call; the pose (J_out, 3).  `last_latency_us` = the
        library's own wall time for it (post start -> pose copied out, no Python overhead)."""
        f = np.ascontiguousarray(np.asarray(frame, dtype=np.float32)).reshape(-1)
        assert f.size == self.st.n_in
        out = np.empty(self.st.n_out, dtype=np.float32)
        lat = ctypes.c_double()
        N.check(self.st._lib.vp3d_stream_serve_step(self.st._s, f.ctypes.data, out.ctypes.data, float(timeout_ms),
                                                    ctypes.byref(lat)), "vp3d_stream_serve_step")
        self.last_latency_us = lat.value
        return out.reshape(-1, 3)

    def __exit__(self, *exc):
        with torch.cuda.device(self.st.device):
            N.check(self.st._lib.vp3d_stream_serve_end(self.st._s, self.stream.cuda_stream), "vp3d_stream_serve_end")
        return False


class _DevBuf:
    """Minimal __cuda_array_interface__ exporter for a raw device pointer."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False),
                                         "version": 2, "strides": None}


def _wrap(ptr: int, n: int, device) -> torch.Tensor:
    with torch.cuda.device(device):
        return torch.as_tensor(_DevBuf(ptr, n), device=device)
