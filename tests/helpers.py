"""Shared test helpers: model construction with synthetic weights."""
import numpy as np
import torch

from vp3d_amd import synth


# 16-bit gates: (max |coordinate delta|, |dMPJPE|) in metres, about 3x the largest error
# measured on MI355X over the lifter tests (round 2: bf16 3.56 mm max on the dilated
# 20,242-frame sequence, 0.057 mm dMPJPE; fp16 0.35 mm at B = 2050, 0.0058 mm), on outputs
# of ~0.11 m rms (synth.normalized_windows inputs): bf16 ~ 9e-2 x rms, fp16 ~ 1.1e-2 x rms.
H16_TOL = {
    "bf16": (1.0e-2, 1.5e-4),
    "fp16": (1.2e-3, 2.0e-5),
}


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
