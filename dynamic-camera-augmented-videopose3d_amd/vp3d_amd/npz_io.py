"""Loading the reference's dataset .npz files without running their pickles.

The reference's datasets are .npz archives whose members are 0-d object arrays
holding nested dicts of numpy arrays (`positions_3d`, `positions_2d`, `cam_seqs`,
`metadata`), read with `np.load(path, allow_pickle=True)` and `.item()`
(run.py:84-87, h36m_dataset.py:235, CMUMocapDataset.py:47-50).  Unpickling with
numpy's loader executes any callable the file names.  Here an object member is
unpickled by an Unpickler whose `find_class` admits only what a pickled tree of
numpy arrays needs: numpy's array reconstructor, `ndarray`, `dtype` (and the numpy 2
dtype classes), and numpy's scalar constructor.  dicts, lists, tuples, strings and
numbers are pickle opcodes, not globals, so nested containers load; any other global
(os.system, builtins.eval, ...) raises `pickle.UnpicklingError` before anything runs.
Plain (non-object) members load through numpy with allow_pickle=False.
"""
from __future__ import annotations

import importlib
import pickle
import zipfile

import numpy as np
from numpy.lib import format as npformat

_ALLOWED = {
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
    ("numpy", "ndarray"), ("numpy", "dtype"),
}


class _ArrayTreeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED:
            mod = module.replace("numpy.core.", "numpy._core.") if hasattr(np, "_core") else module
            return getattr(importlib.import_module(mod), name)
        if module == "numpy.dtypes" and name.endswith("DType") and hasattr(np, "dtypes"):
            return getattr(np.dtypes, name)
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name} (only numpy array trees)")


def _read_member(z: zipfile.ZipFile, name: str):
    with z.open(name) as f:
        version = npformat.read_magic(f)
        if version == (1, 0):
            shape, fortran, dtype = npformat.read_array_header_1_0(f)
        elif version in ((2, 0), (3, 0)):
            shape, fortran, dtype = npformat.read_array_header_2_0(f)
        else:
            raise ValueError(f"{name}: unsupported .npy version {version}")
        if dtype.hasobject:
            return _ArrayTreeUnpickler(f).load()
    with z.open(name) as f:
        return npformat.read_array(f, allow_pickle=False)


def load_npz(path: str) -> dict:
    """{member name: array} of an .npz; object members come back as the ndarray the
    reference's np.load would return (call .item() on 0-d ones)."""
    out = {}
    with zipfile.ZipFile(path) as z:
        for member in z.namelist():
            key = member[:-4] if member.endswith(".npy") else member
            out[key] = _read_member(z, member)
    return out


def load_tree(path: str, key: str):
    """The Python object of member `key` (a 0-d object array's .item())."""
    v = load_npz(path)[key]
    if isinstance(v, np.ndarray) and v.dtype.hasobject and v.shape == ():
        return v.item()
    return v
