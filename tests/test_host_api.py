"""C++ mirror of the reference API (RateLimiter / RateLimitConfig / GpuRateLimiter)."""
import os
import subprocess

import pytest

import rl_amd

BIN = os.path.join(rl_amd.PKG_DIR, "bin", "test_host_api")


def _run(mode):
    if not os.path.exists(BIN):
        subprocess.check_call(["make", "-s", "-C", rl_amd.PKG_DIR])
    r = subprocess.run([BIN, mode], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"{mode}: ok" in r.stdout


def test_host_api_cpu():
    _run("cpu")


@pytest.mark.gpu
def test_host_api_gpu():
    _run("gpu")
