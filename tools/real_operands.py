#!/usr/bin/env python3
"""Real GEMM operands of the Optimized1f stack for tools/ubench/mfma_bias (file mode): the
block-b k3 conv's input rows (3 frames tap-major, as the library's GEMM reads them) and
weights, and the block-b 1x1 conv's input rows (the k3 output after BN + ReLU) and weights,
computed in float64 on the CPU from the synthetic weights (vp3d_amd.synth) and the config-4
windows (or the config-3 dolly windows with --dolly).  Writes raw float32 row-major files.

    python tools/real_operands.py OUTDIR [--block 1] [--rows 1024] [--dolly]
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
import torch.nn.functional as F  # noqa: E402

from helpers import make_model  # noqa: E402
from vp3d_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--block", type=int, default=1)
    ap.add_argument("--rows", type=int, default=1024)
    ap.add_argument("--dolly", action="store_true")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    jin = 23 if a.dolly else 17
    _, sd = make_model(True, jin=jin, channels=1024, seed=0)
    T_b = 3 ** (4 - a.block)  # output rows per window of block b's k3 conv
    B = -(-a.rows // T_b)
    if a.dolly:
        sys.path.insert(0, os.path.join(REPO, "tools"))
        from split_f16_study import dolly_windows
        x = dolly_windows(B)
    else:
        x = synth.normalized_windows(1, "real_operands", B, 243, n_joints=jin)
    t = {k: torch.from_numpy(np.asarray(v)).double() for k, v in sd.items() if not k.endswith("tracked")}

    def bn(h, name):
        return F.batch_norm(h, t[name + ".running_mean"], t[name + ".running_var"], t[name + ".weight"],
                            t[name + ".bias"], False, 0.1, 1e-5)
    with torch.no_grad():
        h = torch.from_numpy(x).double().reshape(B, 243, -1).permute(0, 2, 1)
        h = F.relu(bn(F.conv1d(h, t["expand_conv.weight"], None, stride=3), "expand_bn"))
        for i in range(a.block):
            w = t[f"layers_conv.{2 * i}.weight"]
            if i + 1 == a.block:
                # k3 GEMM rows: output row (b, j) = input frames 3j, 3j+1, 3j+2, tap-major K
                L = h.shape[2] // 3
                A = h[:, :, :3 * L].reshape(B, 1024, L, 3).permute(0, 2, 3, 1).reshape(B * L, 3 * 1024)
                W = w.permute(0, 2, 1).reshape(1024, 3 * 1024)
            res = h[:, :, 1::3]
            h = F.relu(bn(F.conv1d(h, w, None, stride=3), f"layers_bn.{2 * i}"))
            if i + 1 == a.block:
                A1 = h.permute(0, 2, 1).reshape(-1, 1024)
                W1 = t[f"layers_conv.{2 * i + 1}.weight"][:, :, 0]
            h = res + F.relu(bn(F.conv1d(h, t[f"layers_conv.{2 * i + 1}.weight"], None), f"layers_bn.{2 * i + 1}"))
    for name, arr in (("k3_A", A[:a.rows]), ("k3_W", W), ("p_A", A1[:a.rows]), ("p_W", W1)):
        arr.float().contiguous().numpy().tofile(os.path.join(a.out, name + ".bin"))
    print(f"block {a.block}: k3 A {tuple(A[:a.rows].shape)}, 1x1 A {tuple(A1[:a.rows].shape)}; "
          f"A rms {A.pow(2).mean().sqrt():.4f}, zero fraction {(A == 0).double().mean():.3f}")


if __name__ == "__main__":
    main()
