"""Shared test helpers: model construction with synthetic weights."""
import numpy as np
import torch

from vp3d_amd import synth


def make_model(strided, fw=(3, 3, 3, 3, 3), causal=False, channels=1024, jin=17, fin=2, jout=17,
               dense=False, seed=0):
    from common.models.TemporalModel import TemporalModel, TemporalModelOptimized1f
    if strided:
        m = TemporalModelOptimized1f(jin, fin, jout, list(fw), causal=causal, channels=channels)
    else:
        m = TemporalModel(jin, fin, jout, list(fw), causal=causal, channels=channels, dense=dense)
    sd = synth.lifter_state_dict([(k, tuple(v.shape)) for k, v in m.state_dict().items()], seed=seed)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.eval()
    return m, sd


def mpjpe_np(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.mean(np.linalg.norm(a - b, axis=-1)))
