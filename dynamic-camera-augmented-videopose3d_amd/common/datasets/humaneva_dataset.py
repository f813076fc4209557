"""HumanEva-I (drop-in for the reference's common/datasets/humaneva_dataset.py:90-120).

Cameras: the three calibrated views C1-C3 per subject (tables.json, from the reference's
tables humaneva_dataset.py:18-82): resolution 640 x 480, orientation quaternion and
translation (mm -> m), float32 as :95-100 stores them; S4 is uncalibrated (empty
records).  Every calibrated subject is reachable under the split prefixes 'Train/',
'Validate/', 'Unlabeled/Train/', 'Unlabeled/Validate/', 'Unlabeled/' (:103-107).
Positions: data_3d_humaneva.npz `positions_3d` {subject: {action: (T, 15, 3)}} in world
coordinates; 15-joint skeleton.  The reference publishes no focal length or principal
point for these cameras, so their camera records (vp3d_amd.datasets) carry extrinsics
only and the trajectory-conditioned input is refused for this dataset.  Read without
unpickling code (vp3d_amd.npz_io).
"""
import copy

import numpy as np

from common.datasets import tables
from common.datasets.mocap_dataset import MocapDataset
from common.skeleton import Skeleton

SPLIT_PREFIXES = ("Train/", "Validate/", "Unlabeled/Train/", "Unlabeled/Validate/", "Unlabeled/")


def humaneva_skeleton():
    s = tables()["skeletons"]["humaneva"]
    return Skeleton(s["parents"], s["joints_left"], s["joints_right"])


def humaneva_cameras():
    """{prefixed subject: [camera dict] * 3} as humaneva_dataset.py:93-107 builds them."""
    t = tables()
    per_subject = {}
    for subject, cams in copy.deepcopy(t["humaneva_extrinsic"]).items():
        out = []
        for i, cam in enumerate(cams):
            cam.update(copy.deepcopy(t["humaneva_intrinsic"][i]))
            for k, v in cam.items():
                if k not in ("id", "res_w", "res_h"):
                    cam[k] = np.array(v, dtype="float32")
            if "translation" in cam:
                cam["translation"] = cam["translation"] / 1000  # mm -> m
            out.append(cam)
        per_subject[subject] = out
    return {prefix + s: cams for s, cams in per_subject.items() for prefix in SPLIT_PREFIXES}


class HumanEvaDataset(MocapDataset):
    def __init__(self, path):
        from vp3d_amd.npz_io import load_tree
        sk = humaneva_skeleton()
        super().__init__(fps=tables()["fps"]["humaneva"], skeleton_2d=sk, skeleton_3d=sk)
        self._cameras = humaneva_cameras()
        data = load_tree(path, "positions_3d")
        self._data = {}
        for subject, actions in data.items():
            self._data[subject] = {}
            for action_name, positions in actions.items():
                self._data[subject][action_name] = {"positions": positions, "cameras": self._cameras[subject]}
