"""Human3.6M (drop-in for the reference's common/datasets/h36m_dataset.py:209-254).

Cameras: the four calibrated views per subject (tables.json, from the reference's
tables h36m_dataset.py:14-207), normalised as h36m_dataset.py:215-232 does: centre
through normalize_screen_coordinates (float64, stored as float32), focal length
f / res_w * 2, translation mm -> m, and the 9-vector 'intrinsic'
[f(2), c(2), k(3), p(2)].  Positions: data_3d_h36m.npz `positions_3d` (world
coordinates, metres), 32 joints reduced to 17 by removing the static joints, with the
shoulders re-parented to the thorax (:244-252) — which the reference cannot do (Q1:
MocapDataset.remove_joints uses an unset attribute).  The .npz is read without
unpickling code (vp3d_amd.npz_io).
"""
import copy

import numpy as np

from common.datasets import tables
from common.datasets.mocap_dataset import MocapDataset
from common.skeleton import Skeleton


def h36m_skeleton():
    s = tables()["skeletons"]["h36m"]
    return Skeleton(s["parents"], s["joints_left"], s["joints_right"])


def _normalized_center(c, w, h):
    # normalize_screen_coordinates (camera.py:14-18) on the host: float64, then float32
    return (np.asarray(c, dtype=np.float32) / w * 2 - np.array([1, h / w])).astype(np.float32)


def h36m_cameras():
    """{subject: [camera dict] * 4} with the reference's normalisation."""
    t = tables()
    out = {}
    for subject, cams in copy.deepcopy(t["h36m_extrinsic"]).items():
        out[subject] = []
        for i, cam in enumerate(cams):
            cam.update(copy.deepcopy(t["h36m_intrinsic"][i]))
            for k, v in cam.items():
                if k not in ("id", "res_w", "res_h"):
                    cam[k] = np.array(v, dtype="float32")
            cam["center"] = _normalized_center(cam["center"], cam["res_w"], cam["res_h"])
            cam["focal_length"] = cam["focal_length"] / cam["res_w"] * 2
            if "translation" in cam:
                cam["translation"] = cam["translation"] / 1000
            cam["intrinsic"] = np.concatenate((cam["focal_length"], cam["center"], cam["radial_distortion"],
                                               cam["tangential_distortion"]))
            out[subject].append(cam)
    return out


class Human36mDataset(MocapDataset):
    def __init__(self, path, remove_static_joints=True):
        from vp3d_amd.npz_io import load_tree
        sk = h36m_skeleton()
        super().__init__(fps=tables()["fps"]["h36m"], skeleton_2d=sk, skeleton_3d=sk)
        self._cameras = h36m_cameras()
        data = load_tree(path, "positions_3d")
        self._data = {}
        for subject, actions in data.items():
            self._data[subject] = {}
            for action_name, positions in actions.items():
                self._data[subject][action_name] = {"positions": positions, "cameras": self._cameras[subject]}
        if remove_static_joints:
            self.remove_joints(tables()["h36m_static_joints"])  # 32 -> 17 joints
            self._skeleton_3d._parents[11] = 8  # shoulders hang from the thorax
            self._skeleton_3d._parents[14] = 8

    def supports_semi_supervised(self):
        return True
