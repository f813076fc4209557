"""Camera records for the trajectory-conditioned input.

The generators build each frame's conditioning matrix as K @ E_t from
cam['intrinsics'] {'focal_length', 'center'} and cam['extrinsics'] (T, 3, 4)
(reference generators.py:115-125, :180-190) — the CMU format
(CMUMocapDataset.py:53-69,90-96).  The reference's H36M path instead carries one
static camera per view as a 9-vector of intrinsics plus an orientation quaternion
and a translation (h36m_dataset.py:209-232), and its UnchunkedGenerator crashes
indexing it (Q1).  `h36m_camera_record` converts an H36M camera into the CMU record
the generators expect: normalised focal length and centre exactly as
h36m_dataset.py:222-223 computes them, and E_t = [R | -R t] for every frame, where
R is the rotation of qinverse(orientation) — the matrix form of world_to_camera
(camera.py:28-30: qrot(qinverse(q), X - t)).  Host-side (a handful of floats per
camera); the per-frame K @ E and the concat then run on device.
"""
from __future__ import annotations

import numpy as np


def quaternion_to_matrix(q) -> np.ndarray:
    """Rotation matrix of a unit quaternion (w, x, y, z), acting on column vectors:
    R @ v == qrot(q, v) (reference quaternion.py:10-24)."""
    w, x, y, z = (float(v) for v in np.asarray(q, dtype=np.float64))
    n = np.sqrt(w * w + x * x + y * y + z * z)
    w, x, y, z = w / n, x / n, y / n, z / n
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def world_to_camera_extrinsic(orientation, translation) -> np.ndarray:
    """3x4 E with E @ [X; 1] == world_to_camera(X, orientation, translation)."""
    qi = np.asarray(orientation, dtype=np.float64) * np.array([1.0, -1.0, -1.0, -1.0])
    R = quaternion_to_matrix(qi)
    t = np.asarray(translation, dtype=np.float64)
    return np.concatenate([R, (-R @ t)[:, None]], axis=1)


def h36m_camera_record(cam: dict, n_frames: int, normalized: bool = True) -> dict:
    """An H36M camera (keys orientation, translation, focal_length, center and, when
    `normalized` is False, res_w / res_h with pixel focal length and centre and the
    translation in mm) -> {'intrinsics': {...}, 'extrinsics': (n_frames, 3, 4)}."""
    f = np.asarray(cam["focal_length"], dtype=np.float32)
    c = np.asarray(cam["center"], dtype=np.float32)
    t = np.asarray(cam["translation"], dtype=np.float64)
    if not normalized:
        w, h = cam["res_w"], cam["res_h"]
        c = (c / w * 2 - np.array([1, h / w])).astype(np.float32)  # h36m_dataset.py:222
        f = (f / w * 2).astype(np.float32)                           # :223
        t = t / 1000                                                 # :225 (mm -> m)
    E = world_to_camera_extrinsic(cam["orientation"], t)
    return {"intrinsics": {"focal_length": f, "center": c},
            "extrinsics": np.repeat(E[None], n_frames, axis=0)}
