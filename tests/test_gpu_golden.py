"""Native lifter vs the reference's own outputs (golden vectors made by importing
the reference, tests/golden/make_golden.py).

fp32 gate (north star): |MPJPE(native, GT) - MPJPE(reference, GT)| <= 1e-4 mm,
and every coordinate within 1e-5 m of the reference.
"""
import json
import os

import numpy as np
import pytest
import torch

from helpers import H16_TOL, mpjpe_np
from vp3d_amd import synth

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = ["opt1f_243_fp32", "opt1f_243_causal_fp32", "seq_243_fp32", "seq_243_causal_fp32",
         "seq_27_fp32", "traj46_243_fp32", "small_dilated_c64", "small_opt1f_c64",
         "small_dense_c64", "small_causal_c64"]


def build(meta, g):
    from common.models.TemporalModel import TemporalModel, TemporalModelOptimized1f
    if meta["strided"]:
        m = TemporalModelOptimized1f(meta["jin"], 2, 17, meta["fw"], causal=meta["causal"],
                                     channels=meta["channels"])
    else:
        m = TemporalModel(meta["jin"], 2, 17, meta["fw"], causal=meta["causal"],
                          channels=meta["channels"], dense=meta["dense"])
    if any(k.startswith("w/") for k in g.files):
        sd = {k[2:]: g[k] for k in g.files if k.startswith("w/")}
    else:
        sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in m.state_dict().items()],
                                     seed=meta["seed"])
    assert synth.state_dict_sha256(sd) == meta["weights_sha256"]
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return m.eval().cuda()


@pytest.mark.parametrize("dtype", ["fp32", "f16x3"])
@pytest.mark.parametrize("name", CASES)
def test_native_fp32_matches_reference(name, dtype):
    """fp32 and the split-fp16 path (f16x3) under the north-star gate."""
    g = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(g["meta"]))
    m = build(meta, g).set_compute_dtype(dtype)
    with torch.no_grad():
        y = m(torch.from_numpy(g["x"]).cuda()).cpu().numpy()
    ref = g["y"]
    assert y.shape == ref.shape
    gt = synth.gt_poses(3, name, ref.shape[0] * ref.shape[1], 17).reshape(ref.shape)
    d = abs(mpjpe_np(y, gt) - mpjpe_np(ref, gt))
    err = float(np.abs(y - ref).max())
    print(f"{name} {dtype}: max|d|={err:.3e} m dMPJPE={d * 1e3:.3e} mm")
    assert err <= 1e-5
    assert d * 1e3 <= 1e-4


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
def test_native_h16_vs_reference(dtype):
    g = np.load(os.path.join(GOLD, "opt1f_243_fp32.npz"), allow_pickle=False)
    meta = json.loads(str(g["meta"]))
    m = build(meta, g).set_compute_dtype(dtype)
    with torch.no_grad():
        y = m(torch.from_numpy(g["x"]).cuda()).cpu().numpy()
    ref = g["y"]
    gt = synth.gt_poses(3, "h16", ref.shape[0], 17).reshape(ref.shape)
    d = abs(mpjpe_np(y, gt) - mpjpe_np(ref, gt))
    print(f"{dtype}: max|d|={np.abs(y - ref).max():.3e} m dMPJPE={d * 1e3:.3e} mm")
    assert np.abs(y - ref).max() <= H16_TOL[dtype][0]
    assert d <= H16_TOL[dtype][1]
