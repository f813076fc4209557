"""On-device input path: normalisation, camera matrices, window batching, mpjpe.

Device-resident restatement of the reference's data path around the lifter
(SURVEY.md §8(a) rows A10-A14), every step a libvp3d kernel:

  normalize_screen      common/camera.py:14-18   (vp3d_normalize_screen, bit-exact incl. Q6)
  image_coordinates     common/camera.py:21-25   (vp3d_image_coordinates)
  camera_matrices       common/generators.py:115-125, :180-190 (vp3d_camera_matrices, K @ E_t)
  world_to_camera       common/camera.py:28-30   (vp3d_world_to_camera)
  gather_windows        common/generators.py:92-137, :193-198 + CamTransformer.py:187-190
                        (vp3d_gather_windows: edge-clamped windows, optional 12-ch camera concat)
  mpjpe                 common/loss.py:11-17     (vp3d_mpjpe_accumulate, f64 partial sums)

`DeviceSequences` keeps every sequence of a dataset split concatenated in HBM
(2D keypoints, 3D poses, per-frame K·E), so a batch of windows is one gather
launch from a (B, 2) table of (sequence, start frame) pairs.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _native as N


def _dev(device):
    return torch.device(device if device is not None else "cuda")


def _stream(t: torch.Tensor) -> int:
    return N.stream_ptr(t.device)


def _require_cuda(t: torch.Tensor, what: str):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise RuntimeError(f"vp3d: {what} must be a HIP device tensor (no CPU fallback)")


def normalize_screen(x: torch.Tensor, w: int, h: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """X/w*2 - [1, h/w] on device; x (..., 2) float32 cuda.  Result equals the
    reference's float64 result rounded to float32 (what run.py:117 stores)."""
    _require_cuda(x, "x")
    assert x.shape[-1] == 2
    x = x.contiguous().float()
    out = torch.empty_like(x) if out is None else out
    with torch.cuda.device(x.device):
        N.check(N.load().vp3d_normalize_screen(x.data_ptr(), x.numel() // 2, int(w), int(h),
                                               out.data_ptr(), _stream(x)))
    return out


def normalize_screen_f64(x: torch.Tensor, w, h, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """X/w*2 - [1, h/w] on device for float64 keypoints and any (possibly float32,
    non-integral) resolution -- the 3DPW path (ThreeDPWDataset.py:87-103, run.py:117):
    the reference keeps the float64 result, which its generator later casts to float32
    (run.py:458); the kernel computes the float64 expression and rounds once.  h / w is
    evaluated here with the very objects given, so a float32 w, h keep the reference's
    float32 division."""
    _require_cuda(x, "x")
    assert x.shape[-1] == 2
    x = x.contiguous().double()
    out = torch.empty(x.shape, dtype=torch.float32, device=x.device) if out is None else out
    with torch.cuda.device(x.device):
        N.check(N.load().vp3d_normalize_screen_f64(x.data_ptr(), x.numel() // 2, float(w), float(h / w),
                                                   out.data_ptr(), _stream(x)))
    return out


def image_coordinates(x: torch.Tensor, w: int, h: int) -> torch.Tensor:
    _require_cuda(x, "x")
    assert x.shape[-1] == 2
    x = x.contiguous().float()
    out = torch.empty_like(x)
    with torch.cuda.device(x.device):
        N.check(N.load().vp3d_image_coordinates(x.data_ptr(), x.numel() // 2, int(w), int(h),
                                                out.data_ptr(), _stream(x)))
    return out


def camera_matrices(intr: torch.Tensor, frame_seq: torch.Tensor, extr: torch.Tensor,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Per-frame K @ E.  intr (S, 4) f32 [fx, fy, cx, cy]; frame_seq (F,) int32;
    extr (F, 3, 4) float64 -> (F, 3, 4) float32."""
    for t, n in ((intr, "intr"), (frame_seq, "frame_seq"), (extr, "extr")):
        _require_cuda(t, n)
    intr = intr.contiguous().float()
    frame_seq = frame_seq.contiguous().to(torch.int32)
    extr = extr.contiguous().double()
    F = extr.shape[0]
    out = torch.empty((F, 3, 4), dtype=torch.float32, device=extr.device) if out is None else out
    with torch.cuda.device(extr.device):
        N.check(N.load().vp3d_camera_matrices(intr.data_ptr(), frame_seq.data_ptr(), extr.data_ptr(),
                                              F, out.data_ptr(), _stream(extr)))
    return out


def world_to_camera(X: torch.Tensor, R, t) -> torch.Tensor:
    """qrot(qinverse(R), X - t) on device for X (..., 3) float32 cuda; R (4,), t (3,)."""
    _require_cuda(X, "X")
    assert X.shape[-1] == 3
    X = X.contiguous().float()
    Rh = np.ascontiguousarray(np.asarray(R, dtype=np.float32).reshape(4))
    th = np.ascontiguousarray(np.asarray(t, dtype=np.float32).reshape(3))
    out = torch.empty_like(X)
    with torch.cuda.device(X.device):
        N.check(N.load().vp3d_world_to_camera(X.data_ptr(), X.numel() // 3, Rh.ctypes.data,
                                              th.ctypes.data, out.data_ptr(), _stream(X)))
    return out


def mpjpe_sums(pred: torch.Tensor, target: torch.Tensor, acc: Optional[torch.Tensor] = None
               ) -> torch.Tensor:
    """Accumulate [sum ||pred - target||, count] (float64, device) over xyz triples."""
    _require_cuda(pred, "pred")
    _require_cuda(target, "target")
    assert pred.shape == target.shape and pred.shape[-1] == 3
    pred = pred.contiguous().float()
    target = target.contiguous().float()
    if acc is None:
        acc = torch.zeros(2, dtype=torch.float64, device=pred.device)
    with torch.cuda.device(pred.device):
        N.check(N.load().vp3d_mpjpe_accumulate(pred.data_ptr(), target.data_ptr(),
                                               pred.numel() // 3, acc.data_ptr(), _stream(pred)))
    return acc


def project_to_2d(X: torch.Tensor, camera_params: torch.Tensor, linear: bool = False) -> torch.Tensor:
    """H36M projection (vp3d_project_to_2d) of camera-space points X (N, *, 3) with
    per-row intrinsics camera_params (N, 9) -> (N, *, 2)."""
    _require_cuda(X, "X")
    assert X.shape[-1] == 3 and camera_params.dim() == 2 and camera_params.shape[-1] == 9
    assert X.shape[0] == camera_params.shape[0]
    Xc = X.contiguous().float()
    prm = camera_params.to(Xc.device).contiguous().float()
    n = int(X.shape[0])
    per = Xc.numel() // (3 * n) if n else 0
    out = torch.empty((*X.shape[:-1], 2), dtype=torch.float32, device=Xc.device)
    with torch.cuda.device(Xc.device):
        N.check(N.load().vp3d_project_to_2d(Xc.data_ptr(), n, per, prm.data_ptr(), 1 if linear else 0,
                                            out.data_ptr(), _stream(Xc)), "vp3d_project_to_2d")
    return out


def pose_metrics(pred: torch.Tensor, target: torch.Tensor, acc: Optional[torch.Tensor] = None
                 ) -> torch.Tensor:
    """vp3d_pose_metrics over (..., J, 3) poses whose leading axes flatten to frames in
    time order: accumulates (float64, device) [MPJPE, P-MPJPE, N-MPJPE, MPJVE error sums,
    n_frames*J, (n_frames-1)*J]."""
    _require_cuda(pred, "pred")
    _require_cuda(target, "target")
    assert pred.shape == target.shape and pred.shape[-1] == 3
    J = int(pred.shape[-2])
    pred = pred.contiguous().float()
    target = target.contiguous().float()
    if acc is None:
        acc = torch.zeros(6, dtype=torch.float64, device=pred.device)
    with torch.cuda.device(pred.device):
        N.check(N.load().vp3d_pose_metrics(pred.data_ptr(), target.data_ptr(), pred.numel() // (3 * J), J,
                                           acc.data_ptr(), _stream(pred)), "vp3d_pose_metrics")
    return acc


class _MpjpeLoss(torch.autograd.Function):
    """mpjpe as a differentiable loss (run.py:478-485): forward = the native reduction,
    backward = vp3d_mpjpe_backward."""

    @staticmethod
    def forward(ctx, pred, target):
        pred = pred.contiguous().float()
        target = target.contiguous().float()
        ctx.save_for_backward(pred, target)
        acc = mpjpe_sums(pred, target)
        return (acc[0] / acc[1]).float()

    @staticmethod
    def backward(ctx, grad):
        pred, target = ctx.saved_tensors
        g = torch.empty_like(pred)
        grad = grad.contiguous().float()
        with torch.cuda.device(pred.device):
            N.check(N.load().vp3d_mpjpe_backward(pred.data_ptr(), target.data_ptr(), pred.numel() // 3,
                                                 grad.data_ptr(), g.data_ptr(), _stream(pred)),
                    "vp3d_mpjpe_backward")
        return g, None


def mpjpe(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Mean per-joint position error (device scalar, float32 like torch.mean);
    differentiable with respect to `pred` (the training loss, run.py:478)."""
    _require_cuda(pred, "pred")
    _require_cuda(target, "target")
    assert pred.shape == target.shape and pred.shape[-1] == 3
    if pred.requires_grad and torch.is_grad_enabled():
        return _MpjpeLoss.apply(pred, target)
    acc = mpjpe_sums(pred, target)
    return (acc[0] / acc[1]).float()


class DeviceSequences:
    """A set of sequences resident in HBM, concatenated along time.

    poses_2d: list of (T_i, J, 2) arrays (already normalised, as run.py:117 leaves them)
    poses_3d: optional list of (T_i, J3, 3) arrays
    cams:     optional list of dicts with 'intrinsics' {'focal_length', 'center'} and
              'extrinsics' (T_i, 3, 4), as CMUMocapDataset provides them
    """

    def __init__(self, poses_2d: Sequence, poses_3d: Optional[Sequence] = None,
                 cams: Optional[Sequence] = None, device=None):
        dev = _dev(device)
        self.device = dev
        lens = [int(p.shape[0]) for p in poses_2d]
        self.lengths = lens
        self.n_seq = len(lens)
        self.joints_2d = int(poses_2d[0].shape[-2])
        self.f2 = int(np.prod(poses_2d[0].shape[1:]))
        off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        self.seq_off = torch.from_numpy(off).to(dev)
        self.seq_len = torch.tensor(lens, dtype=torch.int32, device=dev)
        self.kps = torch.from_numpy(np.concatenate(
            [np.asarray(p, dtype=np.float32).reshape(p.shape[0], -1) for p in poses_2d])).to(dev)
        self.p3d = None
        if poses_3d is not None:
            self.f3 = int(np.prod(poses_3d[0].shape[1:]))
            self.p3d = torch.from_numpy(np.concatenate(
                [np.asarray(p, dtype=np.float32).reshape(p.shape[0], -1) for p in poses_3d])).to(dev)
        self.cam = None
        if cams is not None:
            intr = np.array([[*c["intrinsics"]["focal_length"], *c["intrinsics"]["center"]]
                             for c in cams], dtype=np.float32)
            fseq = np.repeat(np.arange(self.n_seq, dtype=np.int32), lens)
            extr = np.concatenate([np.asarray(c["extrinsics"], dtype=np.float64) for c in cams])
            self.intr = torch.from_numpy(intr).to(dev)
            self.frame_seq = torch.from_numpy(fseq).to(dev)
            self.extr = torch.from_numpy(extr).to(dev)
            self.cam = torch.empty((extr.shape[0], 12), dtype=torch.float32, device=dev)
            self.refresh_cameras()

    def refresh_cameras(self) -> None:
        """(Re)compute the per-frame K @ E table (vp3d_camera_matrices)."""
        camera_matrices(self.intr, self.frame_seq, self.extr, out=self.cam.view(-1, 3, 4))

    def gather(self, pairs: torch.Tensor, window: int, lead: int, source: str = "2d",
               concat_cams: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Windows of `window` frames starting `lead` frames before each pair's start,
        edge-clamped per sequence.  pairs: (B, 2) int32 device (seq, start).
        source '2d' -> (B, window, F2 [+12]); '3d' -> (B, window, F3); 'cam' -> (B, window, 12)."""
        _require_cuda(pairs, "pairs")
        pairs = pairs.contiguous().to(torch.int32)
        B = int(pairs.shape[0])
        cams_ptr = None
        if source == "2d":
            src, f = self.kps, self.f2
            if concat_cams:
                if self.cam is None:
                    raise ValueError("no cameras loaded")
                cams_ptr = self.cam.data_ptr()
        elif source == "3d":
            src, f = self.p3d, self.f3
        elif source == "cam":
            src, f = self.cam, 12
        else:
            raise ValueError(source)
        fo = f + (12 if cams_ptr else 0)
        if out is None:
            out = torch.empty((B, window, fo), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            N.check(N.load().vp3d_gather_windows(src.data_ptr(), f, cams_ptr, self.seq_off.data_ptr(),
                                                 self.seq_len.data_ptr(), pairs.data_ptr(), B, window,
                                                 int(lead), 0, out.data_ptr(), N.stream_ptr(self.device)))
        return out


class SyntheticWindowPool:
    """The synthetic window source of the bench (configs 2-4) and the 16-bit trajectory
    tests: `n_seq` random-walk 2D keypoint tracks (1280x720 pixels, normalised as
    run.py:117 does) resident in HBM, optionally with per-frame procedural cameras
    (CMU intrinsics, yaw + linear dolly: vp3d_amd.synth.camera_extrinsics), and a seeded
    global table of (sequence, start) pairs.  Identical on every rank, so a global batch
    is sharded by slicing the pair table (vp3d_amd.shard.shard_range) and each rank
    gathers its own windows on device (the ChunkedGenerator gather, generators.py:102-137)."""

    def __init__(self, seed: int, device=None, cameras: bool = False, n_seq: int = 64, seq_len: int = 2048):
        from . import synth
        kps, cams = [], []
        for i in range(n_seq):
            trk = synth.keypoint_tracks(seed, f"pool{i}", seq_len)
            kps.append((trk / 1280 * 2 - np.array([1, 720 / 1280])).astype(np.float32))
            cams.append({"intrinsics": synth.CMU_INTRINSICS,
                         "extrinsics": synth.camera_extrinsics(seed, f"pool{i}", seq_len)})
        self.seqs = DeviceSequences(kps, None, cams if cameras else None, device)
        self.n_seq, self.seq_len, self.seed = n_seq, seq_len, seed

    def global_pairs(self, G: int) -> np.ndarray:
        """(G, 2) int32 (sequence, start frame) table, a pure function of the pool seed."""
        rng = np.random.RandomState(self.seed + 1)
        return np.stack([rng.randint(0, self.n_seq, size=G), rng.randint(0, self.seq_len, size=G)],
                        axis=-1).astype(np.int32)
