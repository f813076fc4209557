"""3DPW with its real moving cameras (drop-in for the reference's
common/datasets/ThreeDPWDataset.py:24-117).

data_3d_3DPW.npz (prepare_data_3dpw.py:58-103) holds three pickled dicts keyed
{subject: {action: ...}}: `positions_3d` (T, 24, 3) SMPL joints in camera space,
`cam_seqs` (T, 3, 4) per-frame extrinsics [R | t] (world -> camera), and `cam_intrinsics`
the 3x3 pixel intrinsics of the sequence.  Every action gets one camera record:

  intrinsics   centre through normalize_screen_coordinates, focal length 2 f / res_w, with
               res_w, res_h = 2 c_x, 2 c_y (:87-103), computed with the reference's numpy
               dtypes so the normalised K is bit-identical;
  extrinsics   the per-frame (T, 3, 4) table, as stored (K.E of generators.py uses it);
  cam_velocity / cam_acceleration / cam_angular_velocity / cam_angular_acceleration
               per-sequence means of the camera-centre motion and of the body angular
               velocity, at the dataset's 60 fps (:60-85): centre c_i = -R_i t_i,
               v = diff(c) fps, a = diff(v) fps, omega_i = vee(log(R_i^T R_{i+1})) fps with
               R_i = E_i[:, :3]^T (the camera-to-world rotation), alpha = diff(omega) fps.
               These feed the PMCC printout of run.py:946-983 (vp3d_amd.evaluate).

The matrix logarithm is the general one (scipy.linalg.logm, as the reference calls it):
3DPW's extrinsics are linearly interpolated 4x (prepare_data_3dpw.py:29-37), so R_i^T
R_{i+1} is not exactly orthogonal and its log has a symmetric part that a closed-form
SO(3) log would drop.  vee reads entries [2,1], [0,2], [1,0] (:8-9).  Skeletons: COCO
(18 joints, 2D) and SMPL (24, 3D), the same trees as CMUMocapDataset's use_3DPW.  Read
without unpickling code (vp3d_amd.npz_io).
"""
import numpy as np

from common.datasets import tables
from common.datasets.mocap_dataset import MocapDataset
from common.skeleton import Skeleton


def _skeleton(name):
    s = tables()["skeletons"][name]
    return Skeleton(s["parents"], s["joints_left"], s["joints_right"])


def _vee(m):
    return np.array([m[2, 1], m[0, 2], m[1, 0]])


def camera_motion(extrinsics, fps):
    """Mean camera velocity, acceleration, angular velocity and angular acceleration of
    one sequence of (T, 3, 4) world -> camera extrinsics (ThreeDPWDataset.py:60-85)."""
    from scipy.linalg import logm

    E = np.asarray(extrinsics)
    R = [e[:, :3].T for e in E]                          # camera -> world rotations
    centres = np.array([-r @ e[:, 3] for r, e in zip(R, E)])  # camera centres in the world
    vel = np.diff(centres, axis=0) * fps
    acc = np.diff(vel, axis=0) * fps
    omega = []
    for i in range(len(R) - 1):
        L = logm(R[i].T @ R[i + 1], disp=False)[0]
        omega.append(_vee(L * fps))
    omega = np.array(omega)
    alpha = np.diff(omega, axis=0) * fps
    return {"cam_velocity": np.mean(vel, axis=0), "cam_acceleration": np.mean(acc, axis=0),
            "cam_angular_velocity": np.mean(omega, axis=0),
            "cam_angular_acceleration": np.mean(alpha, axis=0)}


def threedpw_intrinsics(K):
    """The normalised camera record of a 3x3 pixel intrinsic matrix (:87-103)."""
    K = np.asarray(K)
    res_w, res_h = 2 * K[0, 2], 2 * K[1, 2]
    cam = {"id": "1", "center": K[:2, 2].astype("float32"),
           "focal_length": np.array([K[0, 0], K[1, 1]], dtype="float32"),
           "radial_distortion": np.array([0, 0, 0], dtype="float32"),
           "tangential_distortion": np.array([0, 0], dtype="float32"),
           "res_w": res_w, "res_h": res_h, "azimuth": 0}
    # normalize_screen_coordinates(center, res_w, res_h) with these very numpy scalars
    # (camera.py:14-18: the h / w term keeps their dtype), then the focal length 2 f / w
    cam["center"] = (cam["center"] / res_w * 2 - np.array([1, res_h / res_w])).astype("float32")
    cam["focal_length"] = 2 * cam["focal_length"] / res_w
    return cam


class ThreeDPWDataset(MocapDataset):
    def __init__(self, path, remove_static_joints=True):
        from vp3d_amd.npz_io import load_tree
        fps = tables()["fps"]["3DPW"]
        super().__init__(fps=fps, skeleton_2d=_skeleton("coco"), skeleton_3d=_skeleton("smpl"))
        pose_data = load_tree(path, "positions_3d")
        cam_seqs = load_tree(path, "cam_seqs")
        cam_intrinsics = load_tree(path, "cam_intrinsics")
        self._data, self._cameras = {}, {}
        for subject, actions in pose_data.items():
            self._data[subject], self._cameras[subject] = {}, {}
            for action_name, positions in actions.items():
                seq = cam_seqs[subject][action_name]
                assert len(seq) == positions.shape[0], (
                    f"Number of extrinsics ({len(seq)}) does not match number of frames ({positions.shape[0]}) "
                    f"for subject {subject} action {action_name}")
                cams = {"intrinsics": threedpw_intrinsics(cam_intrinsics[subject][action_name]),
                        "extrinsics": seq}
                cams.update(camera_motion(seq, fps))
                self._data[subject][action_name] = {"positions": positions, "cameras": cams}
                self._cameras[subject][action_name] = cams

    def supports_semi_supervised(self):
        return False
