#!/usr/bin/env python3
"""Where the split-fp16 path's systematic output scale comes from: eps (least-squares scale
of the native output against the fp32 oracle, in units of 2^-24) for Optimized1f stacks of
growing depth, per dtype, on the config-2/4 windows.

    python tools/x3_depth.py [--B 512] [--dtypes fp32,f16x3,fp16]
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

from helpers import make_model  # noqa: E402
from oracle.temporal_ref import lifter_forward  # noqa: E402
from vp3d_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--dtypes", default="fp32,f16x3,fp16")
    ap.add_argument("--channels", type=int, default=1024)
    ap.add_argument("--variants", default="default",
                    help="comma list of default | q64 (VP3D_GEMM=q64) | pack (VP3D_X3_EXPAND=pack) | q64pack")
    args = ap.parse_args()
    envs = {"default": {}, "q64": {"VP3D_GEMM": "q64"}, "pack": {"VP3D_X3_EXPAND": "pack"},
            "q64pack": {"VP3D_GEMM": "q64", "VP3D_X3_EXPAND": "pack"},
            "nosign": {"VP3D_X3_SIGNS": "0"}}
    torch.set_num_threads(16)
    for depth in range(1, 6):
        fw = [3] * depth
        model, sd = make_model(True, fw=fw, channels=args.channels, seed=0)
        model = model.cuda()
        rf = model.receptive_field()
        x = synth.normalized_windows(1, f"depth{depth}", args.B, rf)
        ref = lifter_forward(sd, x, fw, strided=True).numpy().astype(np.float64)
        rr = float(np.sum(ref * ref))
        line = [f"fw={fw} rms {np.sqrt(rr / ref.size):.4f}"]
        for dt in args.dtypes.split(","):
            for var in (args.variants.split(",") if dt == "f16x3" else ["default"]):
                for k in ("VP3D_GEMM", "VP3D_X3_EXPAND", "VP3D_X3_SIGNS"):
                    os.environ.pop(k, None)
                os.environ.update(envs[var])
                # a fresh model per variant: the split weights are made when the lifter uploads them
                model, _ = make_model(True, fw=fw, channels=args.channels, seed=0)
                model = model.cuda()
                model.set_compute_dtype(dt)
                with torch.no_grad():
                    y = model(torch.from_numpy(x).cuda()).cpu().numpy().astype(np.float64)
                d = y - ref
                eps = float(np.sum(d * ref) / rr)
                rel = float(np.sqrt(np.sum(d * d) / rr))
                tag = dt if var == "default" else f"{dt}/{var}"
                line.append(f"{tag}: eps {eps * 2 ** 24:+7.2f} rms {rel * 2 ** 24:7.2f}")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
