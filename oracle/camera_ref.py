"""ORACLE (test infrastructure only): restatement of the reference geometry helpers.

Follows reference common/camera.py:14-34 and common/quaternion.py:10-35.
  normalize_screen_coordinates  X/w*2 - [1, h/w]     (float64 promotion of the offset, quirk Q6)
  image_coordinates             (X + [1, h/w])*w/2
  world_to_camera               qrot(qinverse(R), X - t)   (torch float32, like the reference's wrap)
  camera_to_world               qrot(R, X) + t
"""
from __future__ import annotations

import numpy as np
import torch


def normalize_screen_coordinates(X, w, h):
    assert X.shape[-1] == 2
    return X / w * 2 - np.array([1.0, h / w])


def image_coordinates(X, w, h):
    assert X.shape[-1] == 2
    return (X + np.array([1.0, h / w])) * w / 2


def qrot(q, v):
    """v + 2 (w (u x v) + u x (u x v)) with q = (w, u); torch tensors (*, 4), (*, 3)."""
    assert q.shape[-1] == 4 and v.shape[-1] == 3 and q.shape[:-1] == v.shape[:-1]
    u = q[..., 1:]
    uv = torch.cross(u, v, dim=-1)
    uuv = torch.cross(u, uv, dim=-1)
    return v + 2 * (q[..., :1] * uv + uuv)


def qinverse(q):
    return torch.cat((q[..., :1], -q[..., 1:]), dim=-1)


def world_to_camera(X, R, t):
    qi = qinverse(torch.from_numpy(np.asarray(R)))
    v = torch.from_numpy(np.asarray(X - t))
    q = qi.expand(*v.shape[:-1], 4).contiguous()
    return qrot(q, v).numpy()


def camera_to_world(X, R, t):
    q = torch.from_numpy(np.asarray(R))
    v = torch.from_numpy(np.asarray(X))
    return qrot(q.expand(*v.shape[:-1], 4).contiguous(), v).numpy() + t
