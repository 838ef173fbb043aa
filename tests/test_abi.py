"""The C-ABI library loads and exports every entry point include/mppi.h declares (no GPU needed)."""
import ctypes
import os
import re
import struct

import numpy as np
import pytest

from conftest import REPO


def _declared():
    src = open(os.path.join(REPO, "include", "mppi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mppi_[A-Za-z_0-9]+)\s*\(", src)))


def test_header_declares_the_survey_boundary():
    names = _declared()
    for n in ["mppi_create", "mppi_load_dynamics", "mppi_set_cost", "mppi_solve", "mppi_get_U", "mppi_set_U",
              "mppi_last_error", "mppi_destroy"]:
        assert n in names


def test_library_exports_every_declared_symbol():
    from mppi_hip import _lib as L
    lib = L.load()
    for n in _declared():
        assert hasattr(lib, n), n
    assert sorted(L.EXPORTED) == _declared()
    assert lib.mppi_abi_version() == 4


def test_presets_match_oracle_constants():
    from mppi_hip import _lib as L
    from oracle.mppi_ref import PRESETS
    for name, p in PRESETS.items():
        c = L.preset_config(name)
        assert (c.K, c.H) == (p.K, p.H), name
        assert c.lambda_ == pytest.approx(p.lam) and c.sigma == pytest.approx(p.sigma)
        assert c.ctrl_clamp == pytest.approx(p.ctrl_clamp) and c.U_clamp == pytest.approx(p.U_clamp)
        assert c.norm_eps == pytest.approx(p.norm_eps) and c.shift_fill == pytest.approx(p.shift_fill)
        assert c.terminal_weight == pytest.approx(p.terminal_weight)
        assert c.update_mode == (1 if p.update == "replace" else 0)


def test_errors_are_codes_not_crashes():
    from mppi_hip import _lib as L
    lib = L.load()
    cfg = L.mppi_config()
    assert lib.mppi_preset(b"no_such_preset", ctypes.byref(cfg)) == L.MPPI_E_ARG
    assert b"unknown preset" in lib.mppi_last_error()
    h = ctypes.c_void_p()
    assert lib.mppi_create(None, 0, ctypes.byref(h)) == L.MPPI_E_ARG
    bad = L.preset_config("cartpole_py")
    bad.K = 0
    assert lib.mppi_create(ctypes.byref(bad), 0, ctypes.byref(h)) == L.MPPI_E_ARG
    bad.K = 32769  # past kMaxK (the reduce stages K softmin weights in LDS)
    assert lib.mppi_create(ctypes.byref(bad), 0, ctypes.byref(h)) == L.MPPI_E_ARG
    big = L.preset_config("humanoid_v3")
    big.H = 16384 // big.nu + 1  # nu * H past the U row limit (16384 floats)
    assert lib.mppi_create(ctypes.byref(big), 0, ctypes.byref(h)) == L.MPPI_E_ARG
    assert lib.mppi_solve(None, 1, None, None, None, 0, None, None, 0) == L.MPPI_E_ARG


def test_weight_blob_layout():
    from mppi_hip.nets import pack_blob
    blob = pack_blob(3, [28, 27, 21, 128, 4], {"a.weight": np.ones((2, 3), np.float32)})
    assert blob[:4] == b"MPPW"
    ver, kind = struct.unpack("<II", blob[4:12])
    dims = struct.unpack("<8i", blob[12:44])
    (nt,) = struct.unpack("<I", blob[44:48])
    assert (ver, kind, dims[:5], nt) == (1, 3, (28, 27, 21, 128, 4), 1)
    (ln,) = struct.unpack("<I", blob[48:52])
    assert blob[52:52 + ln] == b"a.weight"
    assert len(blob) == 52 + ln + 4 + 8 + 24
