"""Pin the oracle (and the drop-in module structure) to the reference's own outputs.

The golden vectors in tests/golden/ were produced by importing the reference
(tests/golden/make_golden.py).  Everything here runs on CPU.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import camera_ref, generators_ref, loss_ref
from oracle.temporal_ref import geometry, lifter_forward, receptive_field
from vp3d_amd import synth

GOLD = os.path.join(os.path.dirname(__file__), "golden")
MODEL_CASES = ["opt1f_243_fp32", "opt1f_243_causal_fp32", "seq_243_fp32", "seq_243_causal_fp32",
               "seq_27_fp32", "traj46_243_fp32", "small_dilated_c64", "small_opt1f_c64",
               "small_dense_c64", "small_causal_c64"]


def load(name):
    return np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)


def case_weights(g, meta):
    if any(k.startswith("w/") for k in g.files):
        return {k[2:]: g[k] for k in g.files if k.startswith("w/")}
    keys = list(zip(meta["keys"], [tuple(s) for s in meta["shapes"]]))
    return synth.lifter_state_dict(keys, seed=meta["seed"])


@pytest.mark.parametrize("name", MODEL_CASES)
def test_oracle_matches_reference_model(name):
    g = load(name)
    meta = json.loads(str(g["meta"]))
    sd = case_weights(g, meta)
    assert synth.state_dict_sha256(sd) == meta["weights_sha256"]
    y = lifter_forward(sd, g["x"], meta["fw"], causal=meta["causal"], strided=meta["strided"],
                       dense=meta["dense"]).numpy()
    assert y.shape == g["y"].shape
    np.testing.assert_allclose(y, g["y"], rtol=0, atol=1e-6)
    # same torch build as the golden run -> the restatement is bit-identical
    if torch.__version__ == json.load(open(os.path.join(GOLD, "MANIFEST.json")))["environment"]["torch"]:
        assert np.array_equal(y, g["y"])


@pytest.mark.parametrize("name", MODEL_CASES)
def test_dropin_module_structure(name):
    """The drop-in classes build the reference's parameters, buffers, geometry."""
    from common.models.TemporalModel import TemporalModel, TemporalModelOptimized1f
    meta = json.loads(str(load(name)["meta"]))
    if meta["strided"]:
        m = TemporalModelOptimized1f(meta["jin"], 2, 17, meta["fw"], causal=meta["causal"],
                                     channels=meta["channels"])
    else:
        m = TemporalModel(meta["jin"], 2, 17, meta["fw"], causal=meta["causal"],
                          channels=meta["channels"], dense=meta["dense"])
    sd = m.state_dict()
    assert list(sd.keys()) == meta["keys"]
    assert [list(v.shape) for v in sd.values()] == meta["shapes"]
    assert sum(p.numel() for p in m.parameters()) == meta["n_params"]
    assert m.receptive_field() == meta["receptive_field"]
    assert m.total_causal_shift() == meta["total_causal_shift"]
    assert m.pad == meta["pad"] and m.causal_shift == meta["causal_shift"]
    pad, shift, _ = geometry(meta["fw"], meta["causal"], meta["strided"], meta["dense"])
    assert pad == meta["pad"] and shift == meta["causal_shift"]


def test_receptive_fields():
    assert receptive_field([3, 3, 3, 3, 3]) == 243
    assert receptive_field([3, 3, 3]) == 27
    assert geometry([3, 3, 3, 3, 3], True, False)[1] == [1, 3, 9, 27, 81]
    assert geometry([3, 3, 3, 3, 3], True, True)[1] == [1, 1, 1, 1, 1]


def test_flop_counts():
    from oracle.temporal_ref import conv_flops_per_pose
    assert conv_flops_per_pose([3] * 5, 34, 1024, 17, True) == 352_569_344
    assert conv_flops_per_pose([3] * 5, 46, 1024, 17, True) == 358_541_312
    assert conv_flops_per_pose([3] * 5, 34, 1024, 17, False) == 33_867_776


# ---------------------------------------------------------------- generators
def _gen_inputs():
    g = load("generators")
    meta = json.loads(str(g["meta"]))
    n = len(meta["lens"])
    kps = [g[f"kps{i}"] for i in range(n)]
    p3d = [g[f"p3d{i}"] for i in range(n)]
    cams = [{"intrinsics": dict(synth.CMU_INTRINSICS), "extrinsics": g[f"extr{i}"]} for i in range(n)]
    return g, meta, kps, p3d, cams


@pytest.mark.parametrize("causal", [0, 1])
def test_oracle_unchunked(causal):
    g, meta, kps, p3d, cams = _gen_inputs()
    pad = meta["pad"]
    for j, (bc, b3, b2) in enumerate(generators_ref.unchunked_sequences(cams, p3d, kps, pad,
                                                                       pad if causal else 0)):
        assert np.array_equal(bc.astype(np.float32), g[f"unchunked_c{causal}_cam{j}"])
        assert np.array_equal(b2, g[f"unchunked_c{causal}_2d{j}"])


@pytest.mark.parametrize("causal", [0, 1])
def test_oracle_chunked(causal):
    g, meta, kps, p3d, cams = _gen_inputs()
    pad, B = meta["pad"], meta["batch_size"]
    pairs = generators_ref.shuffled_pairs(meta["lens"], 1, 1234)
    assert np.array_equal(pairs, g[f"chunked_c{causal}_pairs"])
    nb = int(g[f"chunked_c{causal}_num_batches"])
    for bi, (bc, b3, b2) in enumerate(generators_ref.chunked_batches(
            cams, p3d, kps, B, 1, pad, pad if causal else 0)):
        if f"chunked_c{causal}_b{bi}_2d" in g.files:
            assert np.array_equal(b2, g[f"chunked_c{causal}_b{bi}_2d"])
            assert np.array_equal(bc, g[f"chunked_c{causal}_b{bi}_cam"])
            assert np.array_equal(b3, g[f"chunked_c{causal}_b{bi}_3d"])
    assert bi == nb - 1


# ---------------------------------------------------------------- camera / loss
@pytest.mark.parametrize("wh", [(1280, 720), (1000, 1002), (1000, 1000)])
def test_oracle_normalize(wh):
    g = load("camera")
    w, h = wh
    X = g[f"norm_in_{w}x{h}"]
    assert np.array_equal(camera_ref.normalize_screen_coordinates(X, w, h), g[f"norm_out_{w}x{h}"])
    n32 = g[f"norm_out_{w}x{h}"].astype(np.float32)
    assert np.array_equal(camera_ref.image_coordinates(n32, w, h), g[f"img_out_{w}x{h}"])


def test_oracle_world_to_camera():
    g = load("camera")
    out = camera_ref.world_to_camera(g["w2c_X"], g["w2c_R"], g["w2c_t"])
    assert np.array_equal(out, g["w2c_out"])
    back = camera_ref.camera_to_world(g["w2c_out"].astype(np.float32), g["w2c_R"], g["w2c_t"])
    np.testing.assert_allclose(back, g["c2w_out"], atol=0)


def test_oracle_projection():
    g = load("projection")
    assert np.array_equal(camera_ref.project_to_2d(g["X"], g["params"]).numpy(), g["proj"])
    assert np.array_equal(camera_ref.project_to_2d_linear(g["X"], g["params"]).numpy(), g["proj_linear"])


def test_oracle_losses():
    g = load("loss")
    p, t = torch.from_numpy(g["pred"]), torch.from_numpy(g["tgt"])
    assert loss_ref.mpjpe(p, t).item() == float(g["mpjpe"])
    assert loss_ref.n_mpjpe(p, t).item() == float(g["n_mpjpe"])
    p2, t2 = g["pred"].reshape(-1, 17, 3), g["tgt"].reshape(-1, 17, 3)
    np.testing.assert_allclose(loss_ref.p_mpjpe(p2.copy(), t2.copy()), g["p_mpjpe"], rtol=1e-12)
    np.testing.assert_allclose(loss_ref.mean_velocity_error(p2, t2), g["mpjve"], rtol=1e-12)
