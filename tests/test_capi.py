"""The C-ABI library loads and exports every entry point include/vp3d.h declares
(CPU only: no compute calls)."""
import ctypes
import os
import re
import subprocess

import pytest

from vp3d_amd import _native as N

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "vp3d.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(vp3d_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_exported():
    lib = N.load()
    syms = header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(N.EXPORTS) == syms, "vp3d_amd/_native.EXPORTS out of sync with include/vp3d.h"


def test_dynamic_symbol_table():
    out = subprocess.run(["nm", "-D", "--defined-only", N.lib_path()], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (vp3d_[a-z0-9_]+)", out))
    assert set(header_symbols()) <= exported


def test_no_undefined_library_symbols():
    """Every symbol of the library's own namespace resolves inside it: a kernel whose host-side
    compilation fails silently (an AMDGPU inline-asm constraint in a kernel body) leaves its
    launch stub undefined, and the library then fails to load on the GPU box."""
    out = subprocess.run(["nm", "-D", "--undefined-only", N.lib_path()], capture_output=True,
                         text=True, check=True).stdout
    own = [ln for ln in out.splitlines() if "vp3d" in ln]
    assert not own, own


def test_abi_and_weight_count():
    lib = N.load()
    assert lib.vp3d_abi_version() == 1
    cfg = N.make_cfg(17, 2, 17, [3, 3, 3, 3, 3], False, 1024, False, N.VARIANT_STRIDED_1F)
    assert lib.vp3d_weight_count(ctypes.byref(cfg)) == 5 + 10 * 4 + 2
    cfg = N.make_cfg(17, 2, 17, [3, 3, 3], False, 1024, False, N.VARIANT_DILATED)
    assert lib.vp3d_weight_count(ctypes.byref(cfg)) == 27


def test_invalid_config_rejected_without_device():
    lib = N.load()
    cfg = N.make_cfg(17, 2, 17, [3, 4, 3], False, 1024, False, N.VARIANT_DILATED)
    assert lib.vp3d_weight_count(ctypes.byref(cfg)) == -1
    h = ctypes.c_void_p()
    rc = lib.vp3d_create(ctypes.byref(cfg), None, 0, ctypes.byref(h))
    assert rc == N.VP3D_ERR_ASSERT
    assert b"odd filter widths" in lib.vp3d_last_error()
    with pytest.raises(AssertionError):
        N.check(rc)


def test_null_arguments():
    lib = N.load()
    assert lib.vp3d_forward(None, None, 1, 1, None, 0, None) == N.VP3D_ERR_ARG
    assert lib.vp3d_receptive_field(None) == -1
    assert lib.vp3d_destroy(None) == N.VP3D_OK


def test_no_values_spilled_into_accumulator_registers():
    """conv_gemm_a4 owns all 256 AGPRs through inline-asm MFMAs (no per-instruction clobbers),
    so any v_accvgpr_write in its code object is the allocator spilling a VGPR there -- a
    silently corrupted accumulator.  build() refuses such an object; this checks the one the
    library was linked from."""
    from vp3d_amd import build as B
    obj = os.path.join(B.BUILD_DIR, "conv_gemm_a4.hip.o")
    if not os.path.exists(obj):
        pytest.skip("library objects not built here")
    assert B.agpr_writes(obj) == 0
