#!/usr/bin/env python3
"""Dump one forward of the bench's window workload (f16x3 by default) to an .npy file, so two
trees' libraries can be compared bit for bit (run each tree's copy of this script with that
tree on sys.path):  python tools/dump_forward.py OUT.npy [--dtype f16x3] [--batch 4096] [--traj]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "dynamic-camera-augmented-videopose3d_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--dtype", default="f16x3")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--traj", action="store_true")
    a = ap.parse_args()
    import bench
    dev = torch.device("cuda", 0)
    case = bench.WindowsCase(a.traj, a.batch, 0, 1, dev)
    y = torch.empty((case.B, 1, bench.JOINTS, 3), device=dev)
    case.lifter.reserve(case.B, case.RF, a.dtype)
    with torch.no_grad():
        case.make_step(a.dtype, y)()
    torch.cuda.synchronize()
    np.save(a.out, y.cpu().numpy())
    print(f"{a.out}: {tuple(y.shape)} from {case.lifter._lib._name if hasattr(case.lifter._lib, '_name') else 'libvp3d'}")


if __name__ == "__main__":
    main()
