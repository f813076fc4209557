"""Drop-in dataset loaders (reference common/datasets/): Human3.6M and the fork's CMU
procedural-camera dataset, read from the reference's .npz layout without unpickling
code (vp3d_amd.npz_io).  Calibration and skeleton constants: tables.json
(tools/gen_dataset_tables.py)."""
import json
import os

_TABLES = None


def tables():
    global _TABLES
    if _TABLES is None:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tables.json")) as f:
            _TABLES = json.load(f)
    return _TABLES
