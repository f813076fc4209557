#!/usr/bin/env python3
"""Systematic-shrink diagnostic for the split-fp16 path on the config-3 dolly windows.

Runs forward_windows(concat_cams=True) in fp32 and f16x3 on the same seeded windows and
reports, against the fp32 oracle: max |delta|, dMPJPE, and the least-squares scale
eps = sum((y - ref) ref) / sum(ref^2) (a sign-correlated accumulation bias shows as eps < 0
well outside its noise), plus the same for the residual after removing the scale.

    python tools/x3_shrink.py [--B 256]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "dynamic-camera-augmented-videopose3d_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from helpers import make_model, mpjpe_np  # noqa: E402
from oracle.temporal_ref import lifter_forward  # noqa: E402
from vp3d_amd import synth  # noqa: E402
from vp3d_amd.pipeline import SyntheticWindowPool  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--dtypes", default="fp32,f16x3")
    ap.add_argument("--config4", action="store_true", help="the config-2/4 windows instead")
    args = ap.parse_args()
    traj = not args.config4
    model, sd = make_model(True, jin=23 if traj else 17, channels=1024, seed=0)
    model = model.cuda()
    dev = torch.device("cuda", 0)
    pool = SyntheticWindowPool(1000, dev, cameras=traj)
    B = args.B
    pairs = torch.from_numpy(pool.global_pairs(B)).to(dev)
    lifter = model.native_lifter(dev)
    jin = 23 if traj else 17
    with torch.no_grad():
        x = pool.seqs.gather(pairs, 243, 121, "2d", concat_cams=traj).view(B, 243, jin, 2).cpu()
    ref = lifter_forward(sd, x, [3, 3, 3, 3, 3], strided=True).numpy().astype(np.float64)
    gt = synth.gt_poses(3, "dolly_gt", B, 17).reshape(ref.shape)
    rr = float(np.sum(ref * ref))
    print(f"windows {B} traj {traj} output rms {np.sqrt(rr / ref.size):.4f} m")
    for dt in args.dtypes.split(","):
        with torch.no_grad():
            y = lifter.forward_windows(pool.seqs, pairs, 243, 121, concat_cams=traj,
                                       dtype=dt).cpu().numpy().astype(np.float64)
        d = y - ref
        eps = float(np.sum(d * ref) / rr)
        rest = d - eps * ref
        dm = mpjpe_np(y, gt) - mpjpe_np(ref, gt)
        dm_rest = mpjpe_np(ref + rest, gt) - mpjpe_np(ref, gt)
        print(f"{dt:6s} max|d| {np.abs(d).max() * 1e3:.5f} mm  rms|d| {np.sqrt(np.mean(d * d)) * 1e3:.5f} mm  "
              f"dMPJPE {dm * 1e3:+.6f} mm  eps {eps:+.3e} ({eps * 2 ** 24:+.2f} x 2^-24)  "
              f"dMPJPE without the scale {dm_rest * 1e3:+.6f} mm", flush=True)


if __name__ == "__main__":
    main()
