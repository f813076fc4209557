#!/usr/bin/env python3
"""Write the dataset constant tables (camera calibrations, skeleton joint trees) the
drop-in dataset classes read, from the reference's own modules, as JSON data:

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_dataset_tables.py [/root/reference]

Output: dynamic-camera-augmented-videopose3d_amd/common/datasets/tables.json holding
  h36m_intrinsic   the four Human3.6M cameras' pixel intrinsics (h36m_dataset.py:14-59)
  h36m_extrinsic   per subject, the four cameras' orientation quaternion and translation
                   in mm (h36m_dataset.py:61-207); subjects without calibration keep {}
  cmu_intrinsic    the CMU procedural camera (CMUMocapDataset.py:53-62)
  skeletons        parents / joints_left / joints_right of h36m (32 joints),
                   h36m_nonstatic (17), coco (18), smpl (24)  (h36m_dataset.py:13-16,
                   CMUMocapDataset.py:8-25)
  h36m_static_joints  the 15 joints Human36mDataset removes (h36m_dataset.py:245)
  humaneva_intrinsic / humaneva_extrinsic  the three HumanEva cameras (humaneva_dataset.py:18-82)
  skeletons also: humaneva (15) (humaneva_dataset.py:14-16); ThreeDPWDataset.py:11-22
                   defines coco / smpl again, identical to CMUMocapDataset's (asserted)
These are calibration and skeleton DATA of the datasets; no reference code is copied.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
sys.path.insert(0, REF)

import numpy as np  # noqa: E402

from common.datasets import CMUMocapDataset as ref_cmu  # noqa: E402
from common.datasets import h36m_dataset as ref_h36m  # noqa: E402
from common.datasets import humaneva_dataset as ref_he  # noqa: E402
from common.datasets import ThreeDPWDataset as ref_3dpw  # noqa: E402


def skel(s):
    return {"parents": [int(v) for v in s.parents()], "joints_left": [int(v) for v in s.joints_left()],
            "joints_right": [int(v) for v in s.joints_right()]}


def plain(v):
    if isinstance(v, (list, tuple, np.ndarray)):
        return [plain(x) for x in v]
    if isinstance(v, dict):
        return {k: plain(x) for k, x in v.items()}
    if isinstance(v, (np.floating, float)):
        return float(v)
    if isinstance(v, (np.integer, int)):
        return int(v)
    return v


def main():
    assert os.path.realpath(ref_h36m.__file__).startswith(os.path.realpath(REF))
    assert skel(ref_3dpw.coco_skeleton) == skel(ref_cmu.coco_skeleton)
    assert skel(ref_3dpw.smpl_skeleton) == skel(ref_cmu.smpl_skeleton)
    # the CMU camera is a literal inside CMUMocapDataset.__init__ (CMUMocapDataset.py:53-62),
    # not reachable without a data file: its pixel values are restated here
    tables = {
        "h36m_intrinsic": plain(ref_h36m.h36m_cameras_intrinsic_params),
        "h36m_extrinsic": plain(ref_h36m.h36m_cameras_extrinsic_params),
        "cmu_intrinsic": {"id": "1", "center": [640.0, 360.0], "focal_length": [1000.0, 1000.0],
                          "radial_distortion": [0.0, 0.0, 0.0], "tangential_distortion": [0.0, 0.0],
                          "res_w": 1280, "res_h": 720, "azimuth": 0},
        "skeletons": {"h36m": skel(ref_h36m.h36m_skeleton), "h36m_nonstatic": skel(ref_cmu.h36m_skeleton_nonstatic),
                      "coco": skel(ref_cmu.coco_skeleton), "smpl": skel(ref_cmu.smpl_skeleton),
                      "humaneva": skel(ref_he.humaneva_skeleton)},
        "humaneva_intrinsic": plain(ref_he.humaneva_cameras_intrinsic_params),
        "humaneva_extrinsic": plain(ref_he.humaneva_cameras_extrinsic_params),
        "h36m_static_joints": [4, 5, 9, 10, 11, 16, 20, 21, 22, 23, 24, 28, 29, 30, 31],
        "fps": {"h36m": 50, "CMU": 240, "3DPW": 60, "humaneva": 60},
    }
    out = os.path.join(REPO, "dynamic-camera-augmented-videopose3d_amd", "common", "datasets", "tables.json")
    with open(out, "w") as f:
        json.dump(tables, f, indent=1)
    print(out)


if __name__ == "__main__":
    main()
