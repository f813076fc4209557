"""Shared test helpers: model construction with synthetic weights."""
import numpy as np
import torch

from vp3d_amd import synth


# 16-bit gates: (max |coordinate delta|, |dMPJPE|) in metres, 1.6-3x the largest error measured
# on MI355X over the lifter tests (round 4, profiles/r04j_pytest_traj_golden_lifter.txt: bf16
# 3.77 mm max on the dilated 20,242-frame sequence, 0.062 mm dMPJPE; fp16 0.37 mm, 0.0074 mm),
# on outputs of ~0.11 m rms (synth.normalized_windows inputs).
H16_TOL = {
    "bf16": (6.0e-3, 1.25e-4),
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
