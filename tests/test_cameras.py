"""H36M camera records for the trajectory path (vp3d_amd.cameras; quirk Q1): the 3x4
extrinsic reproduces the reference's world_to_camera (restated in the oracle,
pinned by tests/golden/camera.npz)."""
import numpy as np

from oracle import camera_ref
from vp3d_amd import cameras, synth


def test_extrinsic_matches_world_to_camera():
    g = np.load(__file__.replace("test_cameras.py", "golden/camera.npz"))
    X, q, t = g["w2c_X"], g["w2c_R"], g["w2c_t"]
    E = cameras.world_to_camera_extrinsic(q, t)
    Xh = np.concatenate([X.astype(np.float64), np.ones(X.shape[:-1] + (1,))], axis=-1)
    got = Xh @ E.T
    np.testing.assert_allclose(got, g["w2c_out"], atol=2e-5)


def test_quaternion_matrix_is_qrot():
    import torch
    q = synth.normal(8, "q", (4,), 1.0)
    q = q / np.linalg.norm(q)
    v = synth.normal(8, "v", (10, 3), 1.0)
    R = cameras.quaternion_to_matrix(q)
    want = camera_ref.qrot(torch.from_numpy(np.tile(q, (10, 1))), torch.from_numpy(v)).numpy()
    np.testing.assert_allclose(v @ R.T, want, atol=1e-12)


def test_h36m_record_normalisation():
    cam = {"orientation": [0.14, -0.15, -0.75, 0.62], "translation": [1841.1, 4955.3, 1563.4],
           "focal_length": [1145.05, 1143.78], "center": [512.54, 515.45], "res_w": 1000, "res_h": 1002}
    rec = cameras.h36m_camera_record(cam, 5, normalized=False)
    f = rec["intrinsics"]["focal_length"]
    c = rec["intrinsics"]["center"]
    np.testing.assert_allclose(f, np.array([1145.05, 1143.78]) / 1000 * 2, rtol=1e-6)
    # float32 like h36m_dataset.py:222 (.astype('float32'))
    np.testing.assert_allclose(c, camera_ref.normalize_screen_coordinates(np.array([512.54, 515.45]), 1000, 1002),
                               atol=1e-7)
    assert rec["extrinsics"].shape == (5, 3, 4)
    # the camera centre maps to the origin of camera space
    Ec = rec["extrinsics"][0]
    centre = np.array(cam["translation"]) / 1000
    np.testing.assert_allclose(Ec @ np.append(centre, 1.0), 0.0, atol=1e-12)
