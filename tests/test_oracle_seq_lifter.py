"""Oracle of the trajectory lifters (oracle/seq_lifter_ref.py) against the reference's own
eval-mode CoupledTransformer / CoupledLSTM outputs (tests/golden/cam_*.npz): forward on
243-frame windows and sliding_window over a padded sequence."""
import json
import os

import numpy as np
import pytest
import torch

from oracle.seq_lifter_ref import lstm_forward, sliding_windows, transformer_forward

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    g = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(g["meta"]))
    return g, meta, {k[2:]: g[k] for k in g.files if k.startswith("w/")}


def _run(kind, state, meta, x2d, xcam):
    if kind == "transformer":
        return transformer_forward(state, x2d, xcam, meta["n_heads"], meta["num_layers"], len(meta["head_layers"]))
    return lstm_forward(state, x2d, xcam, meta["hidden_size"], meta["num_cells"], len(meta["head_layers"]))


@pytest.mark.parametrize("name,kind", [("cam_transformer", "transformer"), ("cam_lstm", "lstm")])
def test_oracle_matches_reference(name, kind):
    torch.set_num_threads(8)
    g, meta, state = load(name)
    y = _run(kind, state, meta, g["x2d"], g["xcam"]).numpy()
    np.testing.assert_allclose(y, g["y"], atol=2e-6, rtol=0)
    w2, wc = sliding_windows(g["seq2d"], g["seqcam"], meta["window"])
    ys = _run(kind, state, meta, w2, wc).numpy().reshape(g["yseq"].shape)
    np.testing.assert_allclose(ys, g["yseq"], atol=2e-6, rtol=0)
