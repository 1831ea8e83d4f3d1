"""CPU-side checks of the C-ABI boundary: the library builds for gfx950, loads, and
exports every entry point include/rl_engine.h declares (no device calls here)."""
import ctypes
import os
import re

import numpy as np

import rl_amd


def _declared():
    src = open(rl_amd.HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(rl_[a-z_0-9]+)\s*\(", src))
    return names


def test_library_exports_every_declared_symbol():
    L = rl_amd.lib()
    declared = _declared()
    assert declared == set(rl_amd.EXPORTS), declared ^ set(rl_amd.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name


def test_rccl_transport_library_exports():
    """librl_rccl.so (the router's RCCL transport, include/rl_rccl.h) builds and exports it all
    (loading it needs RCCL's runtime, not a GPU)."""
    path = os.path.join(rl_amd.PKG_DIR, "librl_rccl.so")
    src = re.sub(r"/\*.*?\*/", "", open(os.path.join(os.path.dirname(rl_amd.HEADER), "rl_rccl.h")).read(),
                 flags=re.S)
    assert set(re.findall(r"\b(rl_[a-z_0-9]+)\s*\(", src)) == set(rl_amd.RCCL_EXPORTS)
    L = ctypes.CDLL(path)
    for name in rl_amd.RCCL_EXPORTS:
        assert hasattr(L, name), name


def test_abi_version_and_strerror():
    L = rl_amd.lib()
    assert L.rl_abi_version() == 3
    assert rl_amd.strerror(0) == "ok"
    assert "capacity" in rl_amd.strerror(rl_amd.RL_E_CAPACITY) or "full" in rl_amd.strerror(-3)


def test_owner_of_matches_python_mix():
    L = rl_amd.lib()
    keys = np.random.default_rng(1).integers(0, 2**63, 200, dtype=np.uint64)
    for g in (1, 2, 4, 8):
        py = rl_amd.owner_of(keys, g)
        c = np.array([L.rl_owner_of(int(k), 0, g) for k in keys], np.uint32)
        assert np.array_equal(py, c)
        if g > 1:
            assert len(set(py.tolist())) == g


def test_status_codes_match_header():
    hdr = open(rl_amd.HEADER).read()
    for name in ("RL_OK", "RL_E_INVALID_ARG", "RL_E_INVALID_REQUEST", "RL_E_CAPACITY",
                 "RL_E_DEVICE", "RL_E_NOMEM", "RL_E_TOO_LARGE", "RL_E_LIMITERS"):
        m = re.search(rf"#define {name}\s+\(?(-?\d+)\)?", hdr)
        assert int(m.group(1)) == getattr(rl_amd, name)


def test_oracle_constants_match_boundary():
    src = open(os.path.join(os.path.dirname(rl_amd.HEADER), "..", "oracle", "rl_oracle.c")).read()
    assert "#define ORC_REM_UNKNOWN (-1)" in src and "#define ORC_REM_INVALID (-2)" in src
    assert rl_amd.REM_UNKNOWN == -1 and rl_amd.REM_INVALID == -2


def test_device_code_object_is_gfx950():
    data = open(rl_amd.LIB_PATH, "rb").read()
    assert b"gfx950" in data
