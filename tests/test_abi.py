"""CPU checks of the C-ABI boundary: libgvx.so loads without a GPU and exports
every function include/gvx.h declares; the Python mirror fails loudly (no CPU
fallback) when no device is present."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "gvx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gvx_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_core_entry_points():
    syms = declared_symbols()
    for s in ("gvx_create", "gvx_klt", "gvx_klt_fb", "gvx_frame_put", "gvx_klt_fb_batch_dev",
              "gvx_detect", "gvx_preint_integrate", "gvx_preint_factor_eval", "gvx_reproj_eval"):
        assert s in syms


def test_library_exports_every_declared_symbol(gvx_mod):
    lib = ctypes.CDLL(gvx_mod.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, f"libgvx.so lacks {missing}"


def test_version_and_status_strings(gvx_mod):
    L = gvx_mod.lib()
    assert L.gvx_version().decode().startswith("gvx")
    assert L.gvx_status_string(0) == b"ok"
    assert L.gvx_status_string(-5) == b"not found"


def test_params_defaults_match_reference(gvx_mod):
    # tracking.cc:385-388 / tracking.h:113
    p = gvx_mod.KltParams()
    gvx_mod.lib().gvx_klt_params_default(ctypes.byref(p))
    assert (p.win, p.max_level, p.max_iter, p.use_initial_flow) == (21, 3, 30, 1)
    assert p.eps == 0.01 and p.min_eig == np.float32(1e-4)


def test_pyramid_layout(gvx_mod):
    """gvx_pyramid_layout (host only): buildOpticalFlowPyramid's level count rule
    (stop when the next level would be <= winSize), ceil-halved level sizes, 64-byte
    pitches holding the 32-pixel ring, 256-byte aligned levels."""
    lay = gvx_mod.pyramid_layout(1280, 560, 3)
    assert lay["nlev"] == 4 and list(lay["w"]) == [1280, 640, 320, 160] and list(lay["h"]) == [560, 280, 140, 70]
    assert gvx_mod.pyramid_layout(1920, 1200, 4)["nlev"] == 5
    assert gvx_mod.pyramid_layout(100, 60, 3)["nlev"] == 2  # 50x30 -> 25x15 would be <= 21
    for w, h, L in [(1280, 560, 3), (333, 149, 3), (1920, 1200, 4), (22, 22, 5)]:
        lay = gvx_mod.pyramid_layout(w, h, L)
        for l in range(lay["nlev"]):
            assert lay["pitch"][l] % 64 == 0 and lay["pitch"][l] >= lay["w"][l] + 64
            assert lay["off"][l] % 256 == 0
            end = lay["off"][l] + lay["pitch"][l] * (lay["h"][l] + 64)
            nxt = lay["off"][l + 1] if l + 1 < lay["nlev"] else lay["bytes"]
            assert end <= nxt
    with pytest.raises(gvx_mod.GvxError):
        gvx_mod.pyramid_layout(21, 100, 3)


def test_no_cpu_fallback_without_device(gvx_mod):
    import os
    if os.path.exists("/dev/kfd"):
        pytest.skip("device present (the ROCm kernel driver is there)")
    with pytest.raises(gvx_mod.GvxError):
        gvx_mod.Context(0)
