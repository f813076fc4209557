"""Evaluation harness of the FCN path (the part of reference run.py the hot path serves).

Restates run.py:677-774 (`evaluate`) and :906-983 (`run_evaluation`) for the
temporal lifter and the trajectory lifters: per action, an UnchunkedGenerator over
that action's sequences, one model call per sequence (run.py:710-713), Protocol #1 MPJPE accumulated with the
reference's N-weighting (run.py:734-738, x1000 -> mm at :762), plus the
post-path protocols (P-MPJPE :744-747, N-MPJPE :732, MPJVE :750) and the PMCC of
per-sequence error vs camera motion (:946-983).

The loop is device-agnostic: on the GPU box every tensor is on the device and
the model is the native lifter; `metrics` selects the implementations
(`DeviceMetrics` = libvp3d mpjpe kernel + torch-on-device post-path metrics).
Tests drive the same loop with the CPU oracle to check the plumbing.
"""
from __future__ import annotations

from typing import Callable, Dict, Iterable, List, Sequence

import numpy as np
import torch


class DeviceMetrics:
    """All four protocols through libvp3d kernels on the predictions' device: Protocol
    #1 the mpjpe reduction, P-MPJPE / N-MPJPE / MPJVE the vp3d_pose_metrics kernel
    (csrc/metrics.hip).  P-MPJPE and MPJVE are returned as
    numpy float32 scalars like the reference's numpy implementations."""

    def __init__(self):
        from . import pipeline
        self._p = pipeline

    def mpjpe(self, pred: torch.Tensor, gt: torch.Tensor) -> float:
        return float(self._p.mpjpe(pred, gt))

    def n_mpjpe(self, pred: torch.Tensor, gt: torch.Tensor) -> float:
        acc = self._p.pose_metrics(pred, gt)
        return float((acc[2] / acc[4]).float())

    def p_mpjpe(self, pred: torch.Tensor, gt: torch.Tensor):
        acc = self._p.pose_metrics(pred, gt).cpu().numpy()
        return np.float32(acc[1] / acc[4])

    def mpjve(self, pred: torch.Tensor, gt: torch.Tensor):
        acc = self._p.pose_metrics(pred, gt).cpu().numpy()
        return np.float32(acc[3] / acc[5])


def _is_seq_lifter(model) -> bool:
    try:
        from common.models.CamLSTM import CamLSTMBase
        from common.models.CamTransformer import CamTransformerBase
    except ImportError:  # pragma: no cover - the drop-in package is always importable here
        return False
    return isinstance(model, (CamLSTMBase, CamTransformerBase))


def evaluate(generator, model: Callable, metrics, action: str | None = None, verbose: bool = True):
    """One pass over `generator` -- an UnchunkedGenerator, or any iterable of
    (cams, batch_3d, batch_2d, info) with a leading batch axis of 1.  The model call
    follows run.py:710-713: a temporal lifter sees the padded 2D sequence, a trajectory
    lifter (CamLSTMBase / CamTransformerBase) runs sliding_window(inputs_2d, inputs_cam,
    generator.seq_length).  Returns (e1, e2, e3, ev) in mm and per-sequence e1."""
    e1 = e2 = e3 = ev = 0.0
    N = 0
    per_seq: List[float] = []
    infos: List[dict] = []
    motion: List[float] = []
    seq_lifter = _is_seq_lifter(model)
    seq_length = getattr(generator, "seq_length", None)
    if seq_lifter and seq_length is None:
        raise ValueError("a trajectory lifter needs the generator's seq_length (run.py:713)")
    batches = generator.next_epoch() if hasattr(generator, "next_epoch") else generator
    with torch.no_grad():
        for cams, batch_3d, batch_2d, info in batches:
            if seq_lifter:
                pred = model.sliding_window(batch_2d, cams, seq_length)
            else:
                pred = model(batch_2d)
            n = batch_3d.shape[0] * batch_3d.shape[1]
            err = metrics.mpjpe(pred, batch_3d)
            e1 += n * err
            e3 += n * metrics.n_mpjpe(pred, batch_3d)
            # P-MPJPE / MPJVE come back as numpy float32 scalars in the reference
            # (run.py:744-750) and accumulate in float32 under numpy 2 promotion;
            # metrics returning numpy scalars reproduce that exactly
            flat_p = pred.reshape(-1, batch_3d.shape[-2], batch_3d.shape[-1])
            flat_t = batch_3d.reshape(-1, batch_3d.shape[-2], batch_3d.shape[-1])
            e2 += n * metrics.p_mpjpe(flat_p, flat_t)
            ev += n * metrics.mpjve(flat_p, flat_t)
            N += n
            per_seq.append(err)
            infos.append(info)
            # mean per-joint GT displacement per frame (run.py:727-730)
            motion.append(float(torch.linalg.norm(torch.diff(batch_3d.double(), dim=1), dim=-1).mean()))
    # every forward but the last was checked for device-side faults by the next one (the handle
    # refuses a call while a fault is pending); the last one is checked here, before any of
    # these errors is reported (split-K timeout, f16x3 range: RuntimeError)
    sync = getattr(model, "sync_status", None)
    if callable(sync):
        sync()
    res = tuple(float((v / N) * 1000) for v in (e1, e2, e3, ev))  # run.py:762-765 order
    if verbose:
        print("----" + action + "----" if action else "----------")
        print("Protocol #1 Error (MPJPE):", res[0], "mm")
        print("Protocol #2 Error (P-MPJPE):", res[1], "mm")
        print("Protocol #3 Error (N-MPJPE):", res[2], "mm")
        print("Velocity Error (MPJVE):", res[3], "mm")
        print("----------")
    return res, per_seq, infos, motion


PMCC_KEYS = ["cam_velocity", "cam_acceleration", "cam_angular_velocity", "cam_angular_acceleration",
             "pose_motion"]


def camera_motion_pmcc(per_seq_e1: Sequence[float], infos: Sequence[dict],
                       motion: Sequence[float]) -> Dict[str, float]:
    """The reference's "PMCC" printout (run.py:946-971), reproduced as written:
    it stacks [e1, |v_cam|, |a_cam|, |w_cam|, |dw_cam|, pose_motion] per sequence as
    ROWS and calls np.corrcoef with its default rowvar=True, so the printed values
    are correlations between sequence 0's row and sequences 1..5's rows, not between
    the variables (quirk Q9; kept for drop-in output parity, needs >= 6 sequences)."""
    cam = PMCC_KEYS[:4]
    if not infos or any(k not in infos[0] for k in cam) or len(per_seq_e1) < 6:
        return {}
    cols = [np.asarray(per_seq_e1, dtype=np.float64)]
    for k in cam:
        cols.append(np.linalg.norm(np.array([np.asarray(i[k], dtype=np.float64) for i in infos]), axis=1))
    cols.append(np.asarray(motion, dtype=np.float64))
    corr = np.corrcoef(np.stack(cols, axis=1))
    return {k: float(corr[0, i + 1]) for i, k in enumerate(PMCC_KEYS)}
