"""ORACLE (test infrastructure only): restatement of the reference metrics.

Follows reference common/loss.py:
  mpjpe               :11-17  mean Euclidean distance over the last axis
  n_mpjpe             :70-80  scale-aligned mpjpe
  p_mpjpe             :29-68  Procrustes-aligned (numpy SVD), reflection fixed via det sign
  mean_velocity_error :82-91  mpjpe of first differences along axis 0
"""
from __future__ import annotations

import numpy as np
import torch


def mpjpe(pred, target):
    assert pred.shape == target.shape
    return torch.mean(torch.linalg.norm(pred - target, dim=-1))


def n_mpjpe(pred, target):
    assert pred.shape == target.shape
    pp = torch.mean(torch.sum(pred ** 2, dim=3, keepdim=True), dim=2, keepdim=True)
    pt = torch.mean(torch.sum(target * pred, dim=3, keepdim=True), dim=2, keepdim=True)
    return mpjpe((pt / pp) * pred, target)


def p_mpjpe(pred, target):
    assert pred.shape == target.shape
    mx = target.mean(axis=1, keepdims=True)
    my = pred.mean(axis=1, keepdims=True)
    x0, y0 = target - mx, pred - my
    nx = np.sqrt((x0 ** 2).sum(axis=(1, 2), keepdims=True))
    ny = np.sqrt((y0 ** 2).sum(axis=(1, 2), keepdims=True))
    x0 = x0 / nx
    y0 = y0 / ny
    U, s, Vt = np.linalg.svd(np.matmul(x0.transpose(0, 2, 1), y0))
    V = Vt.transpose(0, 2, 1)
    R = np.matmul(V, U.transpose(0, 2, 1))
    sgn = np.sign(np.expand_dims(np.linalg.det(R), axis=1))
    V[:, :, -1] *= sgn
    s[:, -1] *= sgn.flatten()
    R = np.matmul(V, U.transpose(0, 2, 1))
    a = np.expand_dims(s.sum(axis=1, keepdims=True), axis=2) * nx / ny
    t = mx - a * np.matmul(my, R)
    aligned = a * np.matmul(pred, R) + t
    return np.mean(np.linalg.norm(aligned - target, axis=-1))


def mean_velocity_error(pred, target):
    assert pred.shape == target.shape
    return np.mean(np.linalg.norm(np.diff(pred, axis=0) - np.diff(target, axis=0), axis=-1))
