"""ORACLE (test infrastructure only): restatement of the reference geometry helpers.

Follows reference common/camera.py:14-34 and common/quaternion.py:10-35.
  normalize_screen_coordinates  X/w*2 - [1, h/w]     (float64 promotion of the offset, quirk Q6)
  image_coordinates             (X + [1, h/w])*w/2
  world_to_camera               qrot(qinverse(R), X - t)   (torch float32, like the reference's wrap)
  camera_to_world               qrot(R, X) + t
  project_to_2d(_linear)        camera.py:37-90 (H36M distortion model; torch float32)
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


def project_to_2d(X, camera_params):
    """H36M projection with radial (k1..k3) and tangential (p1, p2) distortion,
    reference common/camera.py:37-67; torch float32, the reference's op order:
    XX = clamp(X_xy / X_z, -1, 1); r2 = sum(XX^2); radial = 1 + sum(k * [r2, r2^2, r2^3]);
    tan = sum(p * XX); out = f * (XX * (radial + tan) + p * r2) + c."""
    X = torch.as_tensor(X)
    cp = torch.as_tensor(camera_params)
    assert X.shape[-1] == 3 and cp.dim() == 2 and cp.shape[-1] == 9 and X.shape[0] == cp.shape[0]
    while cp.dim() < X.dim():
        cp = cp.unsqueeze(1)
    f, c, k, p = cp[..., :2], cp[..., 2:4], cp[..., 4:7], cp[..., 7:]
    XX = torch.clamp(X[..., :2] / X[..., 2:], min=-1, max=1)
    r2 = torch.sum(XX ** 2, dim=-1, keepdim=True)
    radial = 1 + torch.sum(k * torch.cat((r2, r2 ** 2, r2 ** 3), dim=-1), dim=-1, keepdim=True)
    tan = torch.sum(p * XX, dim=-1, keepdim=True)
    return f * (XX * (radial + tan) + p * r2) + c


def project_to_2d_linear(X, camera_params):
    """Linear part only (focal length, principal point): camera.py:69-90."""
    X = torch.as_tensor(X)
    cp = torch.as_tensor(camera_params)
    assert X.shape[-1] == 3 and cp.dim() == 2 and cp.shape[-1] == 9 and X.shape[0] == cp.shape[0]
    while cp.dim() < X.dim():
        cp = cp.unsqueeze(1)
    return cp[..., :2] * torch.clamp(X[..., :2] / X[..., 2:], min=-1, max=1) + cp[..., 2:4]
