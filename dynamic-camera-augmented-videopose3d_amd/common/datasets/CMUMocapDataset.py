"""The fork's CMU dataset with procedural per-frame cameras (drop-in for the reference's
common/datasets/CMUMocapDataset.py:27-106).

data_3d_<name>.npz holds `positions_3d` {subject: {action: (T, J, 3)}} (camera space,
prepare_data_cmu_camera.py:60-66) and `cam_seqs` {subject: {action: {cam_extrinsic
(T, 3, 4), cam_velocity, cam_acceleration, cam_angular_velocity,
cam_angular_acceleration, pose_2d_flow}}}.  Every action gets one camera record:
the CMU intrinsics normalised as :63-69 (centre through normalize_screen_coordinates,
focal length 2 f / res_w) and the per-frame extrinsics.  use_3DPW selects the COCO 2D /
SMPL 3D skeletons (:37-39).  Read without unpickling code (vp3d_amd.npz_io).
"""
import copy

import numpy as np

from common.datasets import tables
from common.datasets.mocap_dataset import MocapDataset
from common.skeleton import Skeleton


def _skeleton(name):
    s = tables()["skeletons"][name]
    return Skeleton(s["parents"], s["joints_left"], s["joints_right"])


def cmu_intrinsics():
    """The CMU camera, normalised (CMUMocapDataset.py:53-69)."""
    cam = copy.deepcopy(tables()["cmu_intrinsic"])
    for k in ("center", "focal_length", "radial_distortion", "tangential_distortion"):
        cam[k] = np.array(cam[k], dtype="float32")
    w, h = cam["res_w"], cam["res_h"]
    cam["center"] = (cam["center"] / w * 2 - np.array([1, h / w])).astype("float32")
    cam["focal_length"] = 2 * cam["focal_length"] / w
    return cam


class CMUMocapDataset(MocapDataset):
    def __init__(self, path, use_3DPW=False, remove_static_joints=True):
        from vp3d_amd.npz_io import load_tree
        if use_3DPW:
            sk2, sk3 = _skeleton("coco"), _skeleton("smpl")
        else:
            sk2 = sk3 = _skeleton("h36m_nonstatic")
        super().__init__(fps=tables()["fps"]["CMU"], skeleton_2d=sk2, skeleton_3d=sk3)
        pose_data = load_tree(path, "positions_3d")
        cam_seqs = load_tree(path, "cam_seqs")
        intr = cmu_intrinsics()
        self.cam_intrinsics = np.concatenate((intr["focal_length"], intr["center"], intr["radial_distortion"],
                                              intr["tangential_distortion"]))
        self._data, self._cameras = {}, {}
        for subject, actions in pose_data.items():
            self._data[subject], self._cameras[subject] = {}, {}
            for action_name, positions in actions.items():
                seq = cam_seqs[subject][action_name]
                assert len(seq["cam_extrinsic"]) == positions.shape[0], (
                    f"{len(seq['cam_extrinsic'])} extrinsics for {positions.shape[0]} frames ({subject} {action_name})")
                cams = {"intrinsics": intr, "extrinsics": seq["cam_extrinsic"]}
                for k in ("cam_velocity", "cam_acceleration", "cam_angular_velocity", "cam_angular_acceleration",
                          "pose_2d_flow"):
                    if k in seq:
                        cams[k] = seq[k]
                self._data[subject][action_name] = {"positions": positions, "cameras": cams}
                self._cameras[subject][action_name] = cams
