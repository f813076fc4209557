"""GPU parity of the trajectory lifters: the drop-in
CoupledTransformer / CoupledLSTM on libvp3d.so (vp3d_seq_forward /
vp3d_seq_sliding_window) against the reference's own eval outputs
(tests/golden/cam_*.npz) and the CPU oracle (oracle/seq_lifter_ref.py).

Tolerance: every output coordinate within 1e-5 (f32 on both sides; the GEMMs, the
softmax and the LSTM's transcendental functions round differently from torch-CPU).
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle.seq_lifter_ref import lstm_forward, sliding_windows, transformer_forward
from vp3d_amd import synth

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-5


def _load(name):
    g = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    return g, json.loads(str(g["meta"])), {k[2:]: g[k] for k in g.files if k.startswith("w/")}


def _model(kind, meta, state):
    if kind == "transformer":
        from common.models.CamTransformer import CoupledTransformer
        m = CoupledTransformer(17, 2, 17, 3, meta["d_model"], meta["num_layers"], meta["n_heads"],
                               meta["dim_feedforward"], meta["head_layers"])
        state = dict(state, **{"positional_encoding.pe": m.positional_encoding.pe})
    else:
        from common.models.CamLSTM import CoupledLSTM
        m = CoupledLSTM(17, 2, 17, 3, meta["hidden_size"], meta["num_cells"], meta["head_layers"])
    m.load_state_dict({k: torch.as_tensor(np.asarray(v)) for k, v in state.items()})
    return m.cuda().eval()


def _oracle(kind, state, meta, x2d, xcam):
    if kind == "transformer":
        return transformer_forward(state, x2d, xcam, meta["n_heads"], meta["num_layers"],
                                   len(meta["head_layers"])).numpy()
    return lstm_forward(state, x2d, xcam, meta["hidden_size"], meta["num_cells"], len(meta["head_layers"])).numpy()


CASES = [("cam_transformer", "transformer"), ("cam_lstm", "lstm")]


@pytest.mark.parametrize("name,kind", CASES)
def test_forward_and_sliding_window_match_reference(name, kind):
    g, meta, state = _load(name)
    m = _model(kind, meta, state)
    with torch.no_grad():
        y = m(torch.from_numpy(g["x2d"]).cuda(), torch.from_numpy(g["xcam"]).cuda()).cpu().numpy()
        ys = m.sliding_window(torch.from_numpy(g["seq2d"]).cuda(), torch.from_numpy(g["seqcam"]).cuda(),
                              meta["window"]).cpu().numpy()
    assert y.shape == g["y"].shape and ys.shape == g["yseq"].shape
    print(name, "forward max|d|", np.abs(y - g["y"]).max(), "sliding max|d|", np.abs(ys - g["yseq"]).max())
    np.testing.assert_allclose(y, g["y"], atol=TOL, rtol=0)
    np.testing.assert_allclose(ys, g["yseq"], atol=TOL, rtol=0)


@pytest.mark.parametrize("name,kind", CASES)
def test_long_sequence_sliding_window_vs_oracle(name, kind):
    """A 1,242-frame padded sequence -> 1,000 windows (one per frame, run.py:713)."""
    torch.set_num_threads(16)
    g, meta, state = _load(name)
    m = _model(kind, meta, state)
    L = 1000 + meta["window"] - 1
    s2 = synth.normalized_windows(11, "long", 1, L)
    sc = synth.normal(12, "long/cam", (1, L, 3, 4), std=0.5).astype(np.float32)
    with torch.no_grad():
        ys = m.sliding_window(torch.from_numpy(s2).cuda(), torch.from_numpy(sc).cuda(), meta["window"]).cpu().numpy()
    w2, wc = sliding_windows(s2, sc, meta["window"])
    ref = _oracle(kind, state, meta, w2, wc).reshape(ys.shape)
    print(name, "max|d|", np.abs(ys - ref).max())
    np.testing.assert_allclose(ys, ref, atol=TOL, rtol=0)


def test_errors():
    g, meta, state = _load("cam_lstm")
    m = _model("lstm", meta, state)
    x2, xc = torch.from_numpy(g["x2d"]), torch.from_numpy(g["xcam"])
    with pytest.raises(RuntimeError):
        m.cpu()(x2, xc)
    m.cuda().train()
    with pytest.raises(NotImplementedError):
        m(x2.cuda(), xc.cuda())
    m.eval()
    with pytest.raises(ValueError):
        m.sliding_window(x2[:1].cuda(), xc[:1].cuda(), 500)
    with pytest.raises(AssertionError):
        m(x2.cuda()[..., :1], xc.cuda())
    from common.models.CamLSTM import UncoupledLSTM
    with pytest.raises(NotImplementedError):
        UncoupledLSTM(17, 2, 3, 17, 128, 2, [128])
