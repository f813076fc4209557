"""Drop-in for the reference's ``common/loss.py`` parity metric, on device.

mpjpe (loss.py:11-17) is the metric BASELINE.json names; here it is one libvp3d
reduction kernel (float64 partial sums) over HIP tensors.  The post-path metrics
(n_mpjpe, p_mpjpe, mean_velocity_error: loss.py:29-91) are SURVEY.md §8(f)
"next" rank 1 and live in vp3d_amd.metrics once built.
"""
import torch

from vp3d_amd import pipeline as _P


def mpjpe(predicted, target):
    assert predicted.shape == target.shape
    return _P.mpjpe(predicted, target)
