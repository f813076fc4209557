"""Drop-in for the reference's ``common/loss.py`` parity metric, on device.

mpjpe (loss.py:11-17) is the metric BASELINE.json names; here it is one libvp3d
reduction kernel (float64 partial sums) over HIP tensors.  The post-path metrics
(n_mpjpe, p_mpjpe, mean_velocity_error: loss.py:29-91) run
in one libvp3d kernel as well (vp3d_pose_metrics: per-frame Procrustes by Horn's
quaternion eigenproblem in float64, csrc/metrics.hip).  Like the reference,
p_mpjpe and mean_velocity_error accept the numpy arrays run.py passes them
(run.py:744-750; they are moved to the GPU) and return numpy float32 scalars;
n_mpjpe returns a device tensor.
"""
import numpy as np
import torch

from vp3d_amd import pipeline as _P


def _dev_pair(predicted, target):
    if isinstance(predicted, np.ndarray) or isinstance(target, np.ndarray):
        if not torch.cuda.is_available():
            raise RuntimeError("vp3d: the pose metrics run on the MI355X kernels only (no CPU fallback)")
        predicted = torch.as_tensor(np.asarray(predicted, dtype=np.float32)).cuda()
        target = torch.as_tensor(np.asarray(target, dtype=np.float32)).cuda()
    return predicted, target


def p_mpjpe(predicted, target):
    """Protocol #2 (loss.py:29-68): MPJPE after per-frame rigid alignment; (N, J, 3)."""
    assert predicted.shape == target.shape
    p, t = _dev_pair(predicted, target)
    acc = _P.pose_metrics(p, t).cpu().numpy()
    return np.float32(acc[1] / acc[4])


def n_mpjpe(predicted, target):
    """Protocol #3 (loss.py:70-80): per-frame scale; (B, T, J, 3) tensors."""
    assert predicted.shape == target.shape
    acc = _P.pose_metrics(predicted, target)
    return (acc[2] / acc[4]).float()


def mean_velocity_error(predicted, target):
    """MPJVE (loss.py:82-91): first difference along axis 0; (N, J, 3)."""
    assert predicted.shape == target.shape
    p, t = _dev_pair(predicted, target)
    acc = _P.pose_metrics(p, t).cpu().numpy()
    return np.float32(acc[3] / acc[5])


def mpjpe(predicted, target):
    assert predicted.shape == target.shape
    return _P.mpjpe(predicted, target)
