"""Drop-in device-resident batching for the reference's ``common/generators.py``.

Same class names, constructor arguments and iteration protocol as
Bart-Weil/Dynamic-Camera-Augmented-VideoPose3D common/generators.py
(ChunkedGenerator :11-137, UnchunkedGenerator :140-205); the windows are built in
HBM by one libvp3d gather launch per array instead of a Python loop of numpy
``pad`` calls and 3x3 @ 3x4 matmuls.

Divergences (documented, deliberate):
  * batches are float32 HIP tensors (the reference yields float64 numpy buffers
    that run.py immediately casts to float32 and moves to the GPU);
  * the last, partial batch has exactly the remaining rows — the reference
    yields its whole reused buffer with stale rows from the previous batch
    (SURVEY.md quirk Q2);
  * ``trajectory=True`` additionally fuses the camera-trajectory concat
    (CamTransformer.py:187-190): batch_2d then has J + 6 "joints"
    ([2D keypoints | K·E flattened] viewed as pairs), ready for a 23-joint lifter.
Flip augmentation arguments are accepted and ignored, as in the reference (Q4).
"""
from __future__ import annotations

import numpy as np
import torch

from vp3d_amd.pipeline import DeviceSequences


def _pairs(lengths, chunk_length):
    out = []
    for i, n in enumerate(lengths):
        n_chunks = (n + chunk_length - 1) // chunk_length
        offset = (n_chunks * chunk_length - n) // 2
        b = np.arange(n_chunks + 1) * chunk_length - offset
        out.extend((i, int(b[k]), int(b[k + 1])) for k in range(n_chunks))
    return out


class ChunkedGenerator:
    """Shuffled fixed-length windows around every chunk of every sequence (training batches)."""

    def __init__(self, batch_size, cams, poses_3d, poses_2d,
                 chunk_length, pad=0, causal_shift=0,
                 shuffle=True, random_seed=1234,
                 kps_left=None, kps_right=None, joints_left=None, joints_right=None,
                 endless=False, device=None, trajectory=False):
        assert len(poses_3d) == len(poses_2d), (len(poses_3d), len(poses_2d))
        assert len(cams) == len(poses_2d)
        self.pairs = _pairs([p.shape[0] for p in poses_2d], chunk_length)
        self.seq_length = chunk_length + 2 * pad
        self.chunk_length = chunk_length
        self.num_batches = (len(self.pairs) + batch_size - 1) // batch_size
        self.batch_size = batch_size
        self.random = np.random.RandomState(random_seed)
        self.shuffle = shuffle
        self.pad = pad
        self.causal_shift = causal_shift
        self.endless = endless
        self.state = None
        self.trajectory = trajectory
        self.kps_left, self.kps_right = kps_left, kps_right
        self.joints_left, self.joints_right = joints_left, joints_right
        self.seqs = DeviceSequences(poses_2d, poses_3d, cams, device)
        self.j2 = int(poses_2d[0].shape[-2])
        self.j3 = poses_3d[0].shape[-2:]

    def num_frames(self):
        return self.num_batches * self.batch_size

    def random_state(self):
        return self.random

    def set_random_state(self, random):
        self.random = random

    def next_pairs(self):
        if self.state is not None:
            return self.state
        pairs = self.random.permutation(self.pairs) if self.shuffle else np.array(self.pairs)
        return 0, pairs

    def next_epoch(self):
        while True:
            start_idx, pairs = self.next_pairs()
            dev_pairs = torch.from_numpy(np.ascontiguousarray(
                np.asarray(pairs)[:, :2], dtype=np.int32)).to(self.seqs.device)
            lead = self.pad + self.causal_shift
            for b_i in range(start_idx, self.num_batches):
                p = dev_pairs[b_i * self.batch_size:(b_i + 1) * self.batch_size]
                n = p.shape[0]
                b2 = self.seqs.gather(p, self.seq_length, lead, "2d", concat_cams=self.trajectory)
                bc = self.seqs.gather(p, self.seq_length, lead, "cam")
                b3 = self.seqs.gather(p, self.chunk_length, 0, "3d")
                if self.endless:
                    self.state = (b_i + 1, pairs)
                yield (bc.view(n, self.seq_length, 3, 4),
                       b3.view(n, self.chunk_length, *self.j3),
                       b2.view(n, self.seq_length, -1, 2))
            if self.endless:
                self.state = None
            else:
                return


class UnchunkedGenerator:
    """One whole sequence per batch (B = 1), edge-padded by (pad + shift, pad - shift)."""

    def __init__(self, cams, poses_3d, poses_2d, pad=0, causal_shift=0,
                 kps_left=None, kps_right=None, joints_left=None, joints_right=None,
                 device=None, trajectory=False):
        assert poses_3d is None or len(poses_3d) == len(poses_2d)
        self.kps_left, self.kps_right = kps_left, kps_right
        self.joints_left, self.joints_right = joints_left, joints_right
        self.pad = pad
        self.causal_shift = causal_shift
        self.cams = cams
        self.poses_3d = [] if poses_3d is None else poses_3d
        self.poses_2d = poses_2d
        self.seq_length = 1 + 2 * pad
        self.trajectory = trajectory
        self.seqs = DeviceSequences(poses_2d, poses_3d if poses_3d else None, cams, device)

    def num_frames(self):
        return sum(p.shape[0] for p in self.poses_2d)

    def next_epoch(self):
        dev = self.seqs.device
        lead = self.pad + self.causal_shift
        for idx, n in enumerate(self.seqs.lengths):
            p = torch.tensor([[idx, 0]], dtype=torch.int32, device=dev)
            L = n + 2 * self.pad
            b2 = self.seqs.gather(p, L, lead, "2d", concat_cams=self.trajectory).view(1, L, -1, 2)
            bc = self.seqs.gather(p, L, lead, "cam").view(1, L, 3, 4)
            b3 = None
            if self.seqs.p3d is not None:
                b3 = self.seqs.gather(p, n, 0, "3d").view(1, n, *self.poses_3d[idx].shape[-2:])
            cam = self.cams[idx]
            info = {k: cam[k] for k in ("cam_velocity", "cam_acceleration", "cam_angular_velocity",
                                        "cam_angular_acceleration") if k in cam}
            yield bc, b3, b2, info
