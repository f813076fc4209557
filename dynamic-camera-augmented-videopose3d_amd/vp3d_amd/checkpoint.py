"""Checkpoint loading without arbitrary unpickling.

A run.py checkpoint (reference run.py:563-569) is a dict of 'epoch', 'lr',
'random_state' (the ChunkedGenerator's numpy RandomState), 'optimizer' and
'model_pos'.  torch.load(weights_only=True) rejects the RandomState, and
weights_only=False executes whatever the pickle names.  Here the weights-only
unpickler is opened for exactly the numpy globals a legacy RandomState is rebuilt
from (its MT19937 key array and the bit-generator constructor, which looks the
generator up by name in numpy's own table), so a reference or run.py checkpoint
loads and nothing else can run.  ``trust=True`` (run.py --trust-checkpoint) is the
explicit opt-out for files the user made themselves with other contents.
"""
from __future__ import annotations

import numpy as np
import torch


def _numpy_random_state_globals():
    import numpy.random._pickle as rp
    out = [rp.__randomstate_ctor, rp.__bit_generator_ctor, np.random.MT19937, np.random.RandomState,
           np.ndarray, np.dtype, np.dtypes.UInt32DType]
    try:
        from numpy._core.multiarray import _reconstruct
    except ImportError:  # numpy < 2
        from numpy.core.multiarray import _reconstruct
    out.append(_reconstruct)
    return out


def load_checkpoint(path: str, trust: bool = False, map_location="cpu"):
    """torch.load of a run.py / reference checkpoint.  Weights-only unless `trust`."""
    if trust:
        return torch.load(path, map_location=map_location, weights_only=False)
    try:
        with torch.serialization.safe_globals(_numpy_random_state_globals()):
            return torch.load(path, map_location=map_location, weights_only=True)
    except Exception as e:  # pickle.UnpicklingError and friends
        raise RuntimeError(
            f"{path}: refused by the weights-only loader ({str(e).splitlines()[0][:200]}); pass "
            "--trust-checkpoint to unpickle it fully if you created this file yourself") from e
