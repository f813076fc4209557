"""Portable, seeded synthetic data for the lifter (weights, keypoints, cameras).

The reference ships no checkpoint and no data, and never seeds its weight init
(SURVEY.md quirk Q7), so parity is pinned on weights produced here.  A
counter-based hash (splitmix64 over (seed, tensor name, element index)) makes
every value a pure function of its coordinates: identical on every machine,
numpy version and process, independent of generation order, and cheap to
re-create at full size (the 1024-channel weights are regenerated, not stored).

Distributions follow SURVEY.md §8(d): Kaiming-normal conv weights; BatchNorm
running_mean U(-0.1, 0.1), running_var U(0.5, 2), weight U(0.5, 1.5),
bias U(-0.1, 0.1).
"""
from __future__ import annotations

import hashlib
import math
from collections import OrderedDict

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def _key(seed: int, name: str) -> np.uint64:
    d = hashlib.sha256(f"{int(seed)}/{name}".encode()).digest()
    return np.uint64(int.from_bytes(d[:8], "little"))


def bits(seed: int, name: str, n: int) -> np.ndarray:
    """n pseudo-random uint64 values for (seed, name)."""
    ctr = np.arange(n, dtype=np.uint64)
    return _splitmix64(ctr ^ _splitmix64(np.array([_key(seed, name)], dtype=np.uint64)))


def uniform(seed: int, name: str, shape, low=0.0, high=1.0) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u = (bits(seed, name, n) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return (low + (high - low) * u).reshape(shape)


def normal(seed: int, name: str, shape, std=1.0) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    m = (n + 1) // 2
    u = (bits(seed, name, 2 * m) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    u1 = 1.0 - u[0::2]  # (0, 1]
    u2 = u[1::2]
    r = np.sqrt(-2.0 * np.log(u1))
    z = np.concatenate([r * np.cos(2 * math.pi * u2), r * np.sin(2 * math.pi * u2)])
    # interleave so element i depends only on pair i // 2
    out = np.empty(2 * m)
    out[0::2] = z[:m]
    out[1::2] = z[m:]
    return (std * out[:n]).reshape(shape)


def lifter_state_dict(keys_shapes, seed: int = 0, shrink_gain: float = 0.05):
    """Synthetic state_dict for a TemporalModel / TemporalModelOptimized1f.

    keys_shapes: iterable of (key, shape) in state_dict order (e.g. from
    ``[(k, tuple(v.shape)) for k, v in model.state_dict().items()]``).
    Returns an OrderedDict of float32 numpy arrays (int64 for
    num_batches_tracked)."""
    out = OrderedDict()
    for key, shape in keys_shapes:
        shape = tuple(shape)
        if key.endswith("num_batches_tracked"):
            out[key] = np.zeros(shape, dtype=np.int64)
            continue
        if key.endswith(".weight") and len(shape) == 3:  # Conv1d (Cout, Cin, k)
            fan_in = shape[1] * shape[2]
            std = math.sqrt(2.0 / fan_in)
            if key.startswith("shrink"):
                std = shrink_gain * math.sqrt(1.0 / fan_in)
            out[key] = normal(seed, key, shape, std).astype(np.float32)
        elif key.startswith("shrink") and key.endswith(".bias"):
            out[key] = uniform(seed, key, shape, -0.05, 0.05).astype(np.float32)
        elif key.endswith("running_mean"):
            out[key] = uniform(seed, key, shape, -0.1, 0.1).astype(np.float32)
        elif key.endswith("running_var"):
            out[key] = uniform(seed, key, shape, 0.5, 2.0).astype(np.float32)
        elif key.endswith(".weight"):  # BatchNorm gamma
            out[key] = uniform(seed, key, shape, 0.5, 1.5).astype(np.float32)
        elif key.endswith(".bias"):  # BatchNorm beta
            out[key] = uniform(seed, key, shape, -0.1, 0.1).astype(np.float32)
        else:
            raise KeyError(f"unexpected state_dict key {key}")
    return out


def state_dict_sha256(sd) -> str:
    h = hashlib.sha256()
    for k, v in sd.items():
        a = np.ascontiguousarray(np.asarray(v))
        h.update(k.encode())
        h.update(str(a.dtype).encode())
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def keypoint_tracks(seed: int, name: str, n_frames: int, n_joints: int = 17,
                    width: int = 1280, height: int = 720) -> np.ndarray:
    """Smooth random-walk pixel tracks (n_frames, n_joints, 2), float32 pixels."""
    base = uniform(seed, name + "/base", (1, n_joints, 2), 0.0, 1.0)
    base = base * np.array([width, height]) * 0.6 + np.array([width, height]) * 0.2
    steps = normal(seed, name + "/steps", (n_frames, n_joints, 2), 2.0)
    trk = base + np.cumsum(steps, axis=0)
    trk[..., 0] = np.clip(trk[..., 0], 0, width)
    trk[..., 1] = np.clip(trk[..., 1], 0, height)
    return trk.astype(np.float32)


def normalized_windows(seed: int, name: str, B: int, T: int, n_joints: int = 17) -> np.ndarray:
    """(B, T, n_joints, 2) float32 windows in normalised screen coordinates."""
    base = uniform(seed, name + "/base", (B, 1, n_joints, 2), -0.6, 0.6)
    steps = normal(seed, name + "/steps", (B, T, n_joints, 2), 0.003)
    return (base + np.cumsum(steps, axis=1)).astype(np.float32)


def camera_extrinsics(seed: int, name: str, n_frames: int) -> np.ndarray:
    """Procedural per-frame extrinsics (n_frames, 3, 4) float64: yaw rotation about
    the vertical axis plus a linear dolly."""
    yaw0, yaw_rate = uniform(seed, name + "/yaw", (2,), -0.5, 0.5)
    t0 = uniform(seed, name + "/t0", (3,), -1.0, 1.0) + np.array([0.0, 0.0, 4.0])
    vel = uniform(seed, name + "/vel", (3,), -0.01, 0.01)
    t = np.arange(n_frames, dtype=np.float64)
    yaw = yaw0 + yaw_rate * t / max(n_frames, 1)
    E = np.zeros((n_frames, 3, 4))
    c, s = np.cos(yaw), np.sin(yaw)
    E[:, 0, 0] = c
    E[:, 0, 2] = s
    E[:, 1, 1] = 1.0
    E[:, 2, 0] = -s
    E[:, 2, 2] = c
    E[:, :, 3] = t0[None, :] + vel[None, :] * t[:, None]
    return E


def gt_poses(seed: int, name: str, n_frames: int, n_joints: int = 17) -> np.ndarray:
    """Root-relative synthetic 3D ground truth (n_frames, n_joints, 3), N(0, 0.2 m),
    joint 0 zeroed as run.py:73 does for CMU/3DPW (quirk Q3)."""
    p = normal(seed, name, (n_frames, n_joints, 3), 0.2).astype(np.float32)
    p -= p[:, :1]
    return p


# CMU camera intrinsics after CMUMocapDataset's normalisation
# (CMUMocapDataset.py:53-69): f = 2*1000/1280, c = normalize((640, 360)) = (0, 0).
CMU_INTRINSICS = {"focal_length": np.array([1.5625, 1.5625], dtype=np.float32),
                  "center": np.array([0.0, 0.0], dtype=np.float32),
                  "res_w": 1280, "res_h": 720}


def synthetic_split(n_subjects: int, n_actions: int, frames: int, joints: int, seed: int,
                    normalize) -> dict:
    """A CMU-style evaluation split {subject: {action: {'positions_3d', 'keypoints',
    'cameras'}}}: random-walk 2D tracks normalised with `normalize(X, w, h)` (the
    reference's normalize_screen_coordinates semantics, 1280x720), root-relative 3D
    (run.py:73, quirk Q3), per-frame procedural extrinsics and motion statistics.
    Sequence lengths differ per action/subject (ragged)."""
    data = {}
    for si in range(n_subjects):
        subj = f"S{si + 1}"
        data[subj] = {}
        for ai in range(n_actions):
            name = f"Action{ai} {si}"
            T = frames + 37 * ai + 11 * si
            key = f"{seed}/{subj}/{ai}"
            kps = np.asarray(normalize(keypoint_tracks(seed + 1, key, T, joints), 1280, 720),
                             dtype=np.float32)
            mot = uniform(seed + 4, key, (4, 3), -1.0, 1.0)
            cams = {"intrinsics": CMU_INTRINSICS, "extrinsics": camera_extrinsics(seed + 2, key, T),
                    "cam_velocity": mot[0], "cam_acceleration": mot[1],
                    "cam_angular_velocity": mot[2], "cam_angular_acceleration": mot[3]}
            data[subj][name] = {"positions_3d": gt_poses(seed + 3, key, T, joints),
                                "keypoints": kps, "cameras": cams}
    return data
