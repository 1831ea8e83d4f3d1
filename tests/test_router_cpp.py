"""The C-ABI multi-GPU router (rl_router_*, include/rl_engine.h) driven from C++
(tests/cpp/test_router.cpp): G = 2 / 4 routers on the box's GPU over an in-process
loopback transport, and one rank over the RCCL transport; bit-exact with the oracle."""
import os
import subprocess

import pytest

import rl_amd

BIN = os.path.join(rl_amd.PKG_DIR, "bin", "test_router")

pytestmark = pytest.mark.gpu


def _run(mode):
    r = subprocess.run([BIN, mode], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"{mode}: ok" in r.stdout, r.stdout
    return r.stdout


def test_router_loopback_g2_g4():
    out = _run("loop")
    assert "0 mismatches" in out


def test_router_rccl_world1():
    _run("rccl")
