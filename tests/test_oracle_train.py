"""The training-step oracle (oracle/train_ref.py) against the reference's own training
iterations (tests/golden/train_*.npz, made by make_golden.py `train`: TemporalModel /
TemporalModelOptimized1f in train mode, mpjpe, backward, Adam(amsgrad), two steps)."""
import json
import os

import numpy as np
import pytest
import torch

from oracle.train_ref import TrainLoop

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = ["train_dilated_c64", "train_opt1f_c64", "train_causal_c64", "train_dense_c32"]


def load_case(name):
    g = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(g["meta"]))
    state = {k[2:]: g[k] for k in g.files if k.startswith("w/")}
    return g, meta, state


@pytest.mark.parametrize("name", CASES)
def test_oracle_train_steps_match_reference(name):
    g, meta, state = load_case(name)
    loop = TrainLoop(state, meta["fw"], causal=meta["causal"], strided=meta["strided"], dense=meta["dense"],
                     lr=meta["lr"], amsgrad=meta["amsgrad"], momentum=meta["momentum"])
    for it in range(meta["steps"]):
        y, loss, grads = loop.step(g[f"s{it}/x"], g[f"s{it}/target"])
        np.testing.assert_array_equal(y.numpy(), g[f"s{it}/y"])
        assert float(loss) == float(g[f"s{it}/loss"])
        for k, v in grads.items():
            np.testing.assert_array_equal(v.numpy(), g[f"s{it}/grad/{k}"], err_msg=k)
        st = loop.state()
        for k, v in st.items():
            np.testing.assert_array_equal(v, g[f"s{it}/after/{k}"], err_msg=k)


def test_oracle_dropout_masks_scale_like_torch():
    """Dropout with explicit masks: kept values scaled by the float32 1/(1-p) as
    at::native::dropout's noise.div_(1 - p)."""
    from oracle.train_ref import _mask_cf
    m = np.array([[1, 0], [1, 1], [0, 1]], dtype=np.uint8)  # (B*L, C) with B=1, L=3
    cf = _mask_cf(m, 1, 3).div_(1 - 0.25)
    assert cf.shape == (1, 2, 3)
    assert cf[0, 0, 0].item() == np.float32(1.0) / np.float32(0.75)
    assert cf[0, 1, 0].item() == 0.0
