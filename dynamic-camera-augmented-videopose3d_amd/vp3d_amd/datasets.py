"""Dataset preparation of run.py (reference run.py:47-124), on the MI355X.

`load_dataset` reads the reference's .npz layout — data_3d_<dataset>.npz and
data_2d_<dataset>_<keypoints>.npz in `data_dir` (the reference hard-codes
/vol/bitbucket/bw1222/data/npz, run.py:48,84) — and returns the evaluation split in
run.py's form:

    {subject: {action: {"positions_3d": [(T, J3, 3) per view],
                        "keypoints":    [(T, J2, 2) per view, normalised],
                        "cameras":      [camera record per view]}}}

Per dataset, as run.py:65-124 prepares it:
  CMU / CMU_3DPW / 3DPW
                  positions -= positions[:, :1] (quirk Q3: the root joint becomes 0);
                  one view per action; keypoints normalised with the CMU resolution;
                  the camera record is the dataset's own (normalised K, per-frame E,
                  camera-motion statistics; 3DPW: its per-sequence intrinsics and the
                  motion means of ThreeDPWDataset.py:60-85).  3DPW keypoints are float64
                  with a float32 resolution 2 c_x, 2 c_y: normalised in float64 and
                  rounded once (vp3d_normalize_screen_f64).
  h36m, humaneva  one view per calibrated camera: world_to_camera(positions, R, t)
                  (vp3d_world_to_camera, bit-exact with the reference's torch-CPU qrot),
                  then joints 1.. made root-relative, the root keeping the trajectory;
                  2D tracks longer than the mocap are cut to its length (run.py:101-106);
                  keypoints normalised with each camera's resolution.  The camera record
                  is built from the static calibration (vp3d_amd.cameras.h36m_camera_record:
                  the quirk-Q1 fix — the reference's generators index the H36M 9-vector
                  as a dict and crash), with zero camera motion.  HumanEva's record
                  has extrinsics only (no published intrinsics: `intrinsics.unknown`),
                  so it feeds the 2D-keypoint lifter, not the trajectory-conditioned one.
Normalisation runs on the device (vp3d_normalize_screen: the reference's float64
promotion rounded once to float32, quirk Q6).  Reading never unpickles code
(vp3d_amd.npz_io).
"""
from __future__ import annotations

import os

import numpy as np
import torch

MOTION_KEYS = ("cam_velocity", "cam_acceleration", "cam_angular_velocity", "cam_angular_acceleration")
DATASETS_3D = ("h36m", "humaneva", "CMU", "CMU_3DPW", "3DPW")
MOVING_CAMERA = ("CMU", "CMU_3DPW", "3DPW")  # one view per action, per-frame extrinsics


def _normalize(kps: np.ndarray, w, h, device) -> np.ndarray:
    from .pipeline import normalize_screen, normalize_screen_f64
    out = np.array(kps, dtype=np.float32, copy=True)
    if kps.dtype == np.float64:
        # float64 keypoints (3DPW; resolution 2 c_x / 2 c_y as float32 scalars)
        x = torch.from_numpy(np.ascontiguousarray(kps[..., :2], dtype=np.float64)).to(device)
        out[..., :2] = normalize_screen_f64(x, w, h).cpu().numpy()
    else:
        if not (float(w).is_integer() and float(h).is_integer()):
            raise ValueError(f"float32 keypoints with a non-integral resolution {w} x {h}")
        x = torch.from_numpy(np.ascontiguousarray(kps[..., :2], dtype=np.float32)).to(device)
        out[..., :2] = normalize_screen(x, w, h).cpu().numpy()
    return out


def _world_to_camera(X: np.ndarray, R, t, device) -> np.ndarray:
    from .pipeline import world_to_camera
    x = torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32)).to(device)
    return world_to_camera(x, R, t).cpu().numpy()


def load_dataset(name: str, data_dir: str, keypoints: str = "gt", device=None):
    """(dataset object, prepared split) of the reference's .npz files."""
    from common.datasets.CMUMocapDataset import CMUMocapDataset
    from common.datasets.ThreeDPWDataset import ThreeDPWDataset
    from common.datasets.h36m_dataset import Human36mDataset
    from common.datasets.humaneva_dataset import HumanEvaDataset
    from .cameras import h36m_camera_record, world_to_camera_extrinsic
    from .npz_io import load_npz

    if name not in DATASETS_3D:
        raise SystemExit(f"--dataset {name}: this path reads {', '.join(DATASETS_3D)} or 'synthetic'")
    device = torch.device(device if device is not None else "cuda")
    path3d = os.path.join(data_dir, f"data_3d_{name}.npz")
    path2d = os.path.join(data_dir, f"data_2d_{name}_{keypoints}.npz")
    cmu = name in MOVING_CAMERA
    if name == "3DPW":
        dataset = ThreeDPWDataset(path3d)
    elif cmu:
        dataset = CMUMocapDataset(path3d, use_3DPW=name == "CMU_3DPW")
    elif name == "humaneva":
        dataset = HumanEvaDataset(path3d)
    else:
        dataset = Human36mDataset(path3d)

    # ---- 3D poses in camera space (run.py:65-81) ----
    for subject in dataset.subjects():
        for action, anim in dataset[subject].items():
            if "positions" not in anim:
                continue
            if cmu:
                pos = anim["positions"]
                pos -= pos[:, :1]  # in place, as the reference does: the root joint is zeroed (Q3)
                anim["positions_3d"] = [pos]
            else:
                views = []
                for cam in anim["cameras"]:
                    if "orientation" not in cam:  # HumanEva S4: no calibration (the reference raises here too)
                        raise ValueError(f"{name}: subject {subject} has 3D poses but uncalibrated cameras")
                    p = _world_to_camera(anim["positions"], cam["orientation"], cam["translation"], device)
                    p[:, 1:] -= p[:, :1]  # root keeps the trajectory
                    views.append(p)
                anim["positions_3d"] = views

    # ---- 2D keypoints (run.py:83-124) ----
    arch = load_npz(path2d)
    kp = arch["positions_2d"].item()
    meta = arch["metadata"].item() if "metadata" in arch else {}
    for subject in dataset.subjects():
        assert subject in kp, f"Subject {subject} is missing from the 2D detections dataset"
        for action in dataset[subject].keys():
            assert action in kp[subject], f"Action {action} of subject {subject} is missing from the 2D detections dataset"
            if "positions_3d" not in dataset[subject][action] or cmu:
                continue
            p3 = dataset[subject][action]["positions_3d"]
            for cam_idx in range(len(kp[subject][action])):
                n = p3[cam_idx].shape[0]
                assert kp[subject][action][cam_idx].shape[0] >= n  # some H36M videos have extra frames
                if kp[subject][action][cam_idx].shape[0] > n:
                    kp[subject][action][cam_idx] = kp[subject][action][cam_idx][:n]
            assert len(kp[subject][action]) == len(p3)
    for subject in kp.keys():
        for action in kp[subject]:
            if cmu:
                intr = dataset.cameras()[subject][action]["intrinsics"]
                kp[subject][action] = [_normalize(kp[subject][action], intr["res_w"], intr["res_h"], device)]
            else:
                for cam_idx, kps in enumerate(kp[subject][action]):
                    cam = dataset.cameras()[subject][cam_idx]
                    kp[subject][action][cam_idx] = _normalize(kps, cam["res_w"], cam["res_h"], device)

    # ---- the split in run.py's form, one camera record per view ----
    data = {}
    for subject in dataset.subjects():
        data[subject] = {}
        for action, anim in dataset[subject].items():
            if "positions_3d" not in anim:
                continue
            views_3d = anim["positions_3d"]
            if cmu:
                cam = dataset.cameras()[subject][action]
                rec = {"intrinsics": cam["intrinsics"], "extrinsics": np.asarray(cam["extrinsics"], dtype=np.float64)}
                for k in MOTION_KEYS:
                    rec[k] = np.asarray(cam.get(k, np.zeros(3)), dtype=np.float64)
                cams = [rec]
            else:
                cams = []
                for cam_idx, cam in enumerate(dataset.cameras()[subject]):
                    if "focal_length" in cam:
                        rec = h36m_camera_record(cam, views_3d[cam_idx].shape[0], normalized=True)
                    else:
                        # HumanEva: extrinsics only (the reference has no intrinsics for it)
                        E = world_to_camera_extrinsic(cam["orientation"], cam["translation"])
                        rec = {"intrinsics": {"focal_length": np.ones(2, np.float32),
                                              "center": np.zeros(2, np.float32), "unknown": True},
                               "extrinsics": np.repeat(E[None], views_3d[cam_idx].shape[0], axis=0)}
                    rec["intrinsics"]["res_w"], rec["intrinsics"]["res_h"] = cam["res_w"], cam["res_h"]
                    for k in MOTION_KEYS:
                        rec[k] = np.zeros(3)  # calibrated static cameras
                    cams.append(rec)
            data[subject][action] = {"positions_3d": list(views_3d), "keypoints": list(kp[subject][action]),
                                     "cameras": cams}
    return dataset, data, meta


def downsample(data: dict, stride: int) -> dict:
    """--downsample (run.py:903-910): every stride-th frame of every view.  Divergence,
    on purpose: each camera record's per-frame extrinsics are decimated with the poses
    (the reference slices only the 2D / 3D poses, run.py:175-180, leaving its moving-camera
    K.E tables one frame per ORIGINAL frame, misaligned with the decimated poses)."""
    if stride <= 1:
        return data
    out = {}
    for s, acts in data.items():
        out[s] = {}
        for a, d in acts.items():
            cams = []
            for c in d["cameras"]:
                c = dict(c)
                c["extrinsics"] = c["extrinsics"][::stride]
                cams.append(c)
            out[s][a] = {"positions_3d": [p[::stride] for p in d["positions_3d"]],
                         "keypoints": [k[::stride] for k in d["keypoints"]], "cameras": cams}
    return out
