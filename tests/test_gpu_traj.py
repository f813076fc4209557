"""16-bit parity of the trajectory-conditioned (46-channel) path — config 3.

The model is the reference's TemporalModelOptimized1f with 23 input "joints" (17 keypoint
pairs + the 12 K.E channels as 6 pairs: CamTransformer.py:187-190 concat order), 1024
channels, run through vp3d_forward_windows (the window gather + camera concat fused into
the expand conv's operand loads).  References: the oracle (reference op sequence, fp32) on
the same gathered windows, and the reference's own output in the traj46 golden.

Two input regimes:
  * golden: the traj46_243_fp32 fixture (camera channels of unit scale);
  * dolly:  the bench's config-3 windows (vp3d_amd.pipeline.SyntheticWindowPool: CMU
            intrinsics, a yaw sweep and a linear dolly of up to 0.01 m/frame over 2,048-frame
            sequences, so K.E translations reach ~22 m and the 3D outputs ~2.7 m).

bf16 rounds every operand and activation to 8 mantissa bits: its absolute error scales with
the activations, which the 20-m camera translations inflate.  tools/bf16_error_study.py
(CPU emulation of the native arithmetic) shows the error comes from every layer, not the
expand conv's camera operands alone (keeping the expand exact leaves 15.6 of 19.2 mm), so
fp16 (11 bits, no overflow at these magnitudes) is the 16-bit dtype of config 3.

Gates (max |coordinate delta|, |dMPJPE|), about 3x the MI355X measurement (round 2):
  golden bf16  5 mm,   0.3 mm    measured 1.59 mm, 0.100 mm (4 windows, output rms 0.13 m)
  golden fp16  0.7 mm, 0.02 mm   measured 0.21 mm, 0.0061 mm
  dolly  bf16  refused by vp3d_forward_windows (measured 30.3 mm, 0.477 mm in round 2)
  dolly  fp16  12 mm,  0.33 mm   measured 3.97 mm, 0.108 mm (512 windows, output rms 0.92 m)
  dolly  fp32   0.02 mm, 1e-4 mm (the north-star gate)
  dolly  f16x3  0.02 mm, 1e-4 mm (the north-star gate, as fp32)  measured 0.006 mm max
         (fp32: 0.009 mm), 8e-6 mm dMPJPE (round 4).  Round 3 measured 3e-4 mm: the f16 MFMA
         leaves its f32 accumulator a small offset toward -inf (no sign-correlated error, but
         -1.2..-1.5 x 2^-24 relative on the positive outputs the ReLU keeps,
         tools/ubench/x3_layer_check.hip), which the ReLU turned into a -3.3 x 2^-24 output
         scale over the 5-block stack.  The split weights are now sign-balanced (odd output
         channels carry -W and -scale, so their offset lands on +S): output scale -0.04 x 2^-24
         (tools/x3_depth.py, profiles/r04j_sign_balanced_numerics.txt).
"""
import json
import os

import numpy as np
import pytest
import torch

from helpers import make_model, mpjpe_np
from oracle.temporal_ref import lifter_forward
from vp3d_amd import synth

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
# (max |coordinate delta| m, |dMPJPE| m) per (regime, dtype)
GATES = {
    ("golden", "bf16"): (5.0e-3, 3.0e-4),
    ("golden", "fp16"): (7.0e-4, 2.0e-5),
    ("dolly", "fp16"): (1.2e-2, 3.3e-4),
}


def _model():
    model, sd = make_model(True, jin=23, channels=1024, seed=0)
    return model.cuda(), sd


def _report(y, ref, gt, what):
    err = float(np.abs(y - ref).max())
    d = abs(mpjpe_np(y, gt) - mpjpe_np(ref, gt))
    rms = float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
    print(f"{what}: max|d| {err * 1e3:.3f} mm, dMPJPE {d * 1e3:.4f} mm, output rms {rms:.3f} m, "
          f"max|d|/rms {err / rms:.2e}")
    return err, d


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_traj46_golden_h16(dtype):
    g = np.load(os.path.join(GOLD, "traj46_243_fp32.npz"), allow_pickle=False)
    meta = json.loads(str(g["meta"]))
    model, sd = _model()
    assert synth.state_dict_sha256(sd) == meta["weights_sha256"]
    model.set_compute_dtype(dtype)
    with torch.no_grad():
        y = model(torch.from_numpy(g["x"]).cuda()).cpu().numpy()
    gt = synth.gt_poses(3, "traj46_gt", y.shape[0], 17).reshape(y.shape)
    err, d = _report(y, g["y"], gt, f"traj46 golden {dtype}")
    ce, me = GATES[("golden", dtype)]
    assert err <= ce and d <= me, (err, d)


def test_traj_dolly_bf16_refused():
    """The camera-concat pipeline refuses bf16 (8-bit mantissa on metre-scale K.E)."""
    from vp3d_amd.pipeline import SyntheticWindowPool
    model, _ = _model()
    dev = torch.device("cuda", torch.cuda.current_device())
    pool = SyntheticWindowPool(1000, dev, cameras=True)
    pairs = torch.from_numpy(pool.global_pairs(8)).to(dev)
    lifter = model.native_lifter(dev)
    with pytest.raises(RuntimeError, match="bf16"):
        lifter.forward_windows(pool.seqs, pairs, 243, 121, concat_cams=True, dtype="bf16")


@pytest.mark.parametrize("dtype", ["fp16"])
def test_traj_dolly_windows_h16(dtype):
    """The config-3 bench data: forward_windows(concat_cams=True) on 512 windows of the
    seeded pool vs the fp32 oracle on the same windows."""
    from vp3d_amd.pipeline import SyntheticWindowPool
    model, sd = _model()
    dev = torch.device("cuda", torch.cuda.current_device())
    pool = SyntheticWindowPool(1000, dev, cameras=True)
    B = 512
    pairs = torch.from_numpy(pool.global_pairs(B)).to(dev)
    lifter = model.native_lifter(dev)
    with torch.no_grad():
        y = lifter.forward_windows(pool.seqs, pairs, 243, 121, concat_cams=True, dtype=dtype).cpu().numpy()
        x = pool.seqs.gather(pairs, 243, 121, "2d", concat_cams=True).view(B, 243, 23, 2).cpu()
    ref = lifter_forward(sd, x, [3, 3, 3, 3, 3], strided=True).numpy()
    gt = synth.gt_poses(3, "dolly_gt", B, 17).reshape(ref.shape)
    err, d = _report(y, ref, gt, f"dolly {dtype}")
    ce, me = GATES[("dolly", dtype)]
    assert err <= ce and d <= me, (err, d)


@pytest.mark.parametrize("dtype", ["fp32", "f16x3"])
def test_traj_dolly_windows_fp32(dtype):
    """fp32 and the split-fp16 path on the same windows meet the north-star gate
    (|dMPJPE| <= 1e-4 mm); f16x3 through the split pack kernel's gather + concat."""
    from vp3d_amd.pipeline import SyntheticWindowPool
    model, sd = _model()
    dev = torch.device("cuda", torch.cuda.current_device())
    pool = SyntheticWindowPool(1000, dev, cameras=True)
    B = 64
    pairs = torch.from_numpy(pool.global_pairs(B)).to(dev)
    lifter = model.native_lifter(dev)
    with torch.no_grad():
        y = lifter.forward_windows(pool.seqs, pairs, 243, 121, concat_cams=True, dtype=dtype).cpu().numpy()
        x = pool.seqs.gather(pairs, 243, 121, "2d", concat_cams=True).view(B, 243, 23, 2).cpu()
    ref = lifter_forward(sd, x, [3, 3, 3, 3, 3], strided=True).numpy()
    gt = synth.gt_poses(3, "dolly_gt", B, 17).reshape(ref.shape)
    err, d = _report(y, ref, gt, f"dolly {dtype}")
    assert err <= 2e-5 and d <= 1e-7, (err, d)
