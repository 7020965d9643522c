"""Shared pytest setup: markers, import paths, library builds, GPU context."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ic-gvins_amd")
ORACLE = os.path.join(ROOT, "oracle")
for p in (PKG, ORACLE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X)")


def _ensure_built():
    if not os.path.exists(os.path.join(ORACLE, "liboracle.so")):
        subprocess.run(["make", "-s", "-C", ORACLE], check=True)
    if not os.path.exists(os.path.join(PKG, "gvx", "libgvx.so")):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(PKG, "csrc")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def gvx_mod():
    import gvx
    return gvx


@pytest.fixture(scope="session")
def orc():
    import oracle
    return oracle


@pytest.fixture(scope="session")
def ctx(gvx_mod):
    # torch ships its own HIP runtime: bring it up before libgvx's (as bench.py
    # does), so tests that stage device buffers with torch see the device
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()
    c = gvx_mod.Context(0)
    yield c
    c.close()
