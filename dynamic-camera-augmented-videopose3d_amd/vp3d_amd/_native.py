"""ctypes binding of libvp3d.so (include/vp3d.h).

This is the only place Python touches the native library.  There is no
fallback: if the library is missing or fails to load, every entry point raises
``ImportError`` / ``RuntimeError`` — the MI355X kernels are the product.

torch is imported first on purpose: the HIP runtime it bundles
(libamdhip64.so.7) is then the one libvp3d.so binds to, so both share one
device context and one set of streams.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (loads the HIP runtime libvp3d binds to)

_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libvp3d.so")

VP3D_OK = 0
VP3D_ERR_ASSERT = 1
VP3D_ERR_ARG = 2
VP3D_ERR_HIP = 3
VP3D_ERR_OOM = 4
VP3D_ERR_STATE = 5

VARIANT_DILATED = 0
VARIANT_STRIDED_1F = 1

DTYPE_F32 = 0
DTYPE_BF16 = 1
DTYPE_F16 = 2
DTYPE_F16X3 = 3
DTYPES = {"fp32": DTYPE_F32, "float32": DTYPE_F32, "f32": DTYPE_F32,
          "bf16": DTYPE_BF16, "bfloat16": DTYPE_BF16,
          "fp16": DTYPE_F16, "float16": DTYPE_F16, "f16": DTYPE_F16,
          "f16x3": DTYPE_F16X3}

MAX_BLOCKS = 8

#: every symbol include/vp3d.h declares (checked by tests/test_capi_symbols.py)
EXPORTS = [
    "vp3d_weight_count", "vp3d_create", "vp3d_load_weights", "vp3d_destroy",
    "vp3d_receptive_field", "vp3d_total_causal_shift", "vp3d_out_frames",
    "vp3d_reserve", "vp3d_forward", "vp3d_forward_windows", "vp3d_sync_status", "vp3d_profile_enable",
    "vp3d_layer_count",
    "vp3d_profile_read", "vp3d_profile_reset", "vp3d_profile_layers", "vp3d_normalize_screen",
    "vp3d_normalize_screen_f64", "vp3d_image_coordinates", "vp3d_camera_matrices", "vp3d_world_to_camera",
    "vp3d_gather_windows", "vp3d_mpjpe_accumulate", "vp3d_pose_metrics", "vp3d_project_to_2d", "vp3d_last_error", "vp3d_abi_version",
    "vp3d_build_hash",
    "vp3d_stream_create", "vp3d_stream_reset", "vp3d_stream_io", "vp3d_stream_step",
    "vp3d_stream_frames_seen", "vp3d_stream_graph_capture", "vp3d_stream_graph_launch",
    "vp3d_stream_destroy", "vp3d_stream_persistent", "vp3d_stream_mode", "vp3d_stream_status",
    "vp3d_stream_serve_begin", "vp3d_stream_serve_post", "vp3d_stream_serve_wait", "vp3d_stream_serve_end",
    "vp3d_stream_trace", "vp3d_stream_serve_step",
    "vp3d_trainer_create", "vp3d_trainer_destroy", "vp3d_train_forward", "vp3d_train_backward",
    "vp3d_train_dropout_mask", "vp3d_train_relu_mask", "vp3d_train_layer_rows", "vp3d_adam_step", "vp3d_mpjpe_backward",
    "vp3d_seq_weight_count", "vp3d_seq_create", "vp3d_seq_destroy", "vp3d_seq_forward",
    "vp3d_seq_sliding_window",
]


class vp3d_cfg(ctypes.Structure):
    _fields_ = [
        ("num_joints_in", ctypes.c_int32),
        ("in_features", ctypes.c_int32),
        ("num_joints_out", ctypes.c_int32),
        ("n_widths", ctypes.c_int32),
        ("filter_widths", ctypes.c_int32 * MAX_BLOCKS),
        ("causal", ctypes.c_int32),
        ("channels", ctypes.c_int32),
        ("dense", ctypes.c_int32),
        ("variant", ctypes.c_int32),
        ("bn_eps", ctypes.c_float),
    ]


SEQ_TRANSFORMER = 0
SEQ_LSTM = 1
SEQ_MAX_HEAD = 8


class vp3d_seq_cfg(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("num_joints_in", ctypes.c_int32),
        ("in_features", ctypes.c_int32),
        ("num_joints_out", ctypes.c_int32),
        ("out_features", ctypes.c_int32),
        ("d_model", ctypes.c_int32),
        ("num_layers", ctypes.c_int32),
        ("n_heads", ctypes.c_int32),
        ("dim_feedforward", ctypes.c_int32),
        ("n_head_layers", ctypes.c_int32),
        ("head_layers", ctypes.c_int32 * SEQ_MAX_HEAD),
        ("max_len", ctypes.c_int32),
        ("eps", ctypes.c_float),
    ]


_lib = None
_lock = threading.Lock()

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_int = ctypes.c_int

_SIGNATURES = {
    "vp3d_weight_count": (_int, [ctypes.POINTER(vp3d_cfg)]),
    "vp3d_create": (_int, [ctypes.POINTER(vp3d_cfg), ctypes.POINTER(_vp), _int, ctypes.POINTER(_vp)]),
    "vp3d_load_weights": (_int, [_vp, ctypes.POINTER(_vp), _int]),
    "vp3d_destroy": (_int, [_vp]),
    "vp3d_receptive_field": (_int, [_vp]),
    "vp3d_total_causal_shift": (_int, [_vp]),
    "vp3d_out_frames": (_int, [_vp, _int]),
    "vp3d_reserve": (_int, [_vp, _int, _int, _int]),
    "vp3d_forward": (_int, [_vp, _vp, _int, _int, _vp, _int, _vp]),
    "vp3d_forward_windows": (_int, [_vp, _vp, _i32, _vp, _vp, _vp, _vp, _int, _int, _int, _vp, _int, _vp]),
    "vp3d_profile_enable": (_int, [_vp, _int]),
    "vp3d_sync_status": (_int, [_vp, _vp]),
    "vp3d_layer_count": (_int, [_vp]),
    "vp3d_profile_read": (_int, [_vp, _vp, _vp, _vp]),
    "vp3d_profile_reset": (_int, [_vp]),
    "vp3d_profile_layers": (_int, [_vp, ctypes.c_uint64]),
    "vp3d_normalize_screen": (_int, [_vp, _i64, _i32, _i32, _vp, _vp]),
    "vp3d_normalize_screen_f64": (_int, [_vp, _i64, ctypes.c_double, ctypes.c_double, _vp, _vp]),
    "vp3d_image_coordinates": (_int, [_vp, _i64, _i32, _i32, _vp, _vp]),
    "vp3d_camera_matrices": (_int, [_vp, _vp, _vp, _i64, _vp, _vp]),
    "vp3d_world_to_camera": (_int, [_vp, _i64, _vp, _vp, _vp, _vp]),
    "vp3d_gather_windows": (_int, [_vp, _i32, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp]),
    "vp3d_mpjpe_accumulate": (_int, [_vp, _vp, _i64, _vp, _vp]),
    "vp3d_mpjpe_backward": (_int, [_vp, _vp, _i64, _vp, _vp, _vp]),
    "vp3d_pose_metrics": (_int, [_vp, _vp, _i64, _i32, _vp, _vp]),
    "vp3d_project_to_2d": (_int, [_vp, _i64, _i64, _vp, _i32, _vp, _vp]),
    "vp3d_stream_create": (_int, [_vp, _int, ctypes.POINTER(_vp)]),
    "vp3d_stream_reset": (_int, [_vp, _vp]),
    "vp3d_stream_io": (_int, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_int)]),
    "vp3d_stream_step": (_int, [_vp, _vp, _vp, _vp]),
    "vp3d_stream_frames_seen": (ctypes.c_int64, [_vp]),
    "vp3d_stream_graph_capture": (_int, [_vp, _vp, _int]),
    "vp3d_stream_graph_launch": (_int, [_vp, _vp]),
    "vp3d_stream_destroy": (_int, [_vp]),
    "vp3d_stream_persistent": (_int, [_vp]),
    "vp3d_stream_mode": (_int, [_vp]),
    "vp3d_stream_status": (_int, [_vp]),
    "vp3d_stream_serve_begin": (_int, [_vp, _vp, ctypes.c_double]),
    "vp3d_stream_serve_post": (_int, [_vp, _vp, ctypes.POINTER(_i64)]),
    "vp3d_stream_serve_wait": (_int, [_vp, _i64, _vp, ctypes.c_double]),
    "vp3d_stream_serve_end": (_int, [_vp, _vp]),
    "vp3d_stream_trace": (_int, [_vp, _vp, ctypes.c_int64, _vp, _vp, _vp]),
    "vp3d_stream_serve_step": (_int, [_vp, _vp, _vp, ctypes.c_double, _vp]),
    "vp3d_trainer_create": (_int, [ctypes.POINTER(vp3d_cfg), ctypes.POINTER(_vp)]),
    "vp3d_trainer_destroy": (_int, [_vp]),
    "vp3d_train_forward": (_int, [_vp, ctypes.POINTER(_vp), _int, _vp, _int, _int, ctypes.c_float,
                                  ctypes.c_double, ctypes.c_uint64, _vp, _vp]),
    "vp3d_train_backward": (_int, [_vp, ctypes.POINTER(_vp), _int, _vp, ctypes.POINTER(_vp), _vp]),
    "vp3d_train_dropout_mask": (_int, [_vp, _int, _i64, _vp, _vp]),
    "vp3d_train_relu_mask": (_int, [_vp, _int, _i64, _vp, _vp]),
    "vp3d_train_layer_rows": (_i64, [_vp, _int]),
    "vp3d_adam_step": (_int, [_int, ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                              ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_i64),
                              ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                              ctypes.c_double, _i64, _int, _vp]),
    "vp3d_seq_weight_count": (_int, [ctypes.POINTER(vp3d_seq_cfg)]),
    "vp3d_seq_create": (_int, [ctypes.POINTER(vp3d_seq_cfg), ctypes.POINTER(_vp), _int, ctypes.POINTER(_vp)]),
    "vp3d_seq_destroy": (_int, [_vp]),
    "vp3d_seq_forward": (_int, [_vp, _vp, _vp, _int, _int, _vp, _vp]),
    "vp3d_seq_sliding_window": (_int, [_vp, _vp, _vp, _int, _int, _vp, _vp]),
    "vp3d_last_error": (ctypes.c_char_p, []),
    "vp3d_abi_version": (_int, []),
    "vp3d_build_hash": (ctypes.c_char_p, []),
}


def lib_path() -> str:
    return _LIB_PATH


def load():
    """Load libvp3d.so (once) and declare every signature.  Raises if missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(_LIB_PATH):
            raise ImportError(
                f"vp3d: native library not built ({_LIB_PATH}); run "
                "`python __graft_entry__.py build` (hipcc --offload-arch=gfx950)")
        lib = ctypes.CDLL(_LIB_PATH, mode=ctypes.RTLD_LOCAL)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _check_provenance(lib)
        _lib = lib
        return lib


def _check_provenance(lib) -> None:
    """The library must have been built from the sources beside it (when they are
    present, as in the repository and its snapshot on the GPU box)."""
    from . import build as _build
    if not os.path.isdir(_build.CSRC):
        return
    want = _build.source_hash()
    got = lib.vp3d_build_hash().decode()
    if got != want:
        raise ImportError(
            f"vp3d: {_LIB_PATH} was built from other sources or for another target (library {got[:16]}, "
            f"tree {want[:16]} for arch {_build.ARCH}, VP3D_OFFLOAD_ARCH); "
            "rebuild with `python __graft_entry__.py build`")


class NativeError(RuntimeError):
    pass


def check(rc: int, what: str = "") -> None:
    """Map a vp3d status code onto the reference's exception convention."""
    if rc == VP3D_OK:
        return
    msg = load().vp3d_last_error().decode("utf-8", "replace")
    if what:
        msg = f"{what}: {msg}"
    if rc == VP3D_ERR_ASSERT:
        raise AssertionError(msg)
    raise NativeError(f"vp3d error {rc}: {msg}")


def make_cfg(num_joints_in, in_features, num_joints_out, filter_widths, causal, channels,
             dense, variant, bn_eps=1e-5) -> vp3d_cfg:
    fw = list(filter_widths)
    if len(fw) > MAX_BLOCKS:
        raise AssertionError(f"at most {MAX_BLOCKS} filter widths are supported")
    cfg = vp3d_cfg()
    cfg.num_joints_in = num_joints_in
    cfg.in_features = in_features
    cfg.num_joints_out = num_joints_out
    cfg.n_widths = len(fw)
    for i, w in enumerate(fw):
        cfg.filter_widths[i] = int(w)
    cfg.causal = 1 if causal else 0
    cfg.channels = channels
    cfg.dense = 1 if dense else 0
    cfg.variant = variant
    cfg.bn_eps = bn_eps
    return cfg


def stream_ptr(device=None) -> int:
    """Raw hipStream_t of torch's current stream on `device`."""
    return torch.cuda.current_stream(device).cuda_stream
