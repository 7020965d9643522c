"""ctypes binding of liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference path (see gvx_oracle.h for what each
function restates and the parity status: unpinned against real OpenCV/Eigen
binaries, pinned by analytic known-answer tests).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")


class KltParams(C.Structure):
    _fields_ = [("win", C.c_int), ("max_level", C.c_int), ("max_iter", C.c_int), ("eps", C.c_double),
                ("use_initial_flow", C.c_int), ("min_eig", C.c_float)]

    @classmethod
    def default(cls, **kw):
        p = cls(21, 3, 30, 0.01, 1, 1e-4)
        for k, v in kw.items():
            setattr(p, k, v)
        return p


class U8Plane(C.Structure):
    _fields_ = [("w", C.c_int), ("h", C.c_int), ("pad", C.c_int), ("pitch", C.c_int),
                ("buf", C.POINTER(C.c_uint8))]


class Pyramid(C.Structure):
    _fields_ = [("nlevels", C.c_int), ("lv", U8Plane * 8)]


class DetectParams(C.Structure):
    _fields_ = [("block_size", C.c_double), ("max_features", C.c_int), ("quality", C.c_double),
                ("subpix_win", C.c_int), ("subpix_iters", C.c_int), ("subpix_eps", C.c_double)]

    @classmethod
    def default(cls, **kw):
        p = cls(200.0, 150, 0.01, 5, 20, 0.01)
        for k, v in kw.items():
            setattr(p, k, v)
        return p


class BlockGrid(C.Structure):
    _fields_ = [("block_cols", C.c_int), ("block_rows", C.c_int), ("block_cnts", C.c_int),
                ("col", C.c_int), ("row", C.c_int), ("max_block_features", C.c_int),
                ("min_pixel_distance", C.c_int)]


class ImuParams(C.Structure):
    _fields_ = [(k, C.c_double) for k in ("acc_vrw", "gyr_arw", "gyr_bias_std", "acc_bias_std",
                                           "corr_time", "gravity")]


class State(C.Structure):
    _fields_ = [("time", C.c_double), ("p", C.c_double * 3), ("q", C.c_double * 4),
                ("v", C.c_double * 3), ("bg", C.c_double * 3), ("ba", C.c_double * 3)]


class Preint(C.Structure):
    _fields_ = [("variant", C.c_int), ("m", C.c_int), ("delta_time", C.c_double),
                ("start_time", C.c_double), ("end_time", C.c_double), ("current", State),
                ("delta", State), ("gravity", C.c_double * 3), ("jacobian", C.c_double * 225),
                ("covariance", C.c_double * 225), ("noise", C.c_double * 144), ("q0", C.c_double * 4),
                ("iewn", C.c_double * 3), ("pn", C.POINTER(C.c_double))]


class ReprojConst(C.Structure):
    _fields_ = [("pts0", C.c_double * 3), ("pts1", C.c_double * 3), ("vel0", C.c_double * 3),
                ("vel1", C.c_double * 3), ("td0", C.c_double), ("td1", C.c_double),
                ("std", C.c_double)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.orc_build_pyramid.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(Pyramid)]
        L.orc_build_pyramid.restype = C.c_int
        L.orc_free_pyramid.argtypes = [C.POINTER(Pyramid)]
        L.orc_scharr.argtypes = [C.POINTER(U8Plane), P]
        L.orc_calc_optical_flow_pyr_lk.argtypes = [P, P, C.c_int, C.c_int, C.c_int, P, P, P, P, C.c_int,
                                                   C.POINTER(KltParams), C.c_int]
        L.orc_klt_fb.argtypes = [P, P, C.c_int, C.c_int, C.c_int, P, P, P, P, P, P, P, C.c_int,
                                 C.c_double, C.c_double, C.c_int, C.c_int, C.POINTER(KltParams),
                                 C.c_int, C.c_int]
        L.orc_klt_fb.restype = C.c_int
        L.orc_block_grid_make.argtypes = [C.c_int, C.c_int, C.POINTER(DetectParams), C.POINTER(BlockGrid)]
        L.orc_mask_circles.argtypes = [P, C.c_int, C.c_int, P, C.c_int, C.c_int]
        L.orc_corner_min_eigen_val.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                               C.c_int, P]
        L.orc_good_features_to_track.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                                 C.c_int, P, C.c_int, C.c_int, C.c_double, C.c_double, P]
        L.orc_good_features_to_track.restype = C.c_int
        L.orc_corner_subpix.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_int,
                                        C.c_int, C.c_int, C.c_double]
        L.orc_features_detection.argtypes = [P, C.c_int, C.c_int, C.c_int, P, C.c_int, P, C.c_int, C.c_int,
                                             C.c_int, C.POINTER(DetectParams), P, P]
        L.orc_features_detection.restype = C.c_int
        L.orc_preint_integrate.argtypes = [C.POINTER(Preint), C.c_int, C.POINTER(ImuParams), P, C.c_int,
                                           C.POINTER(State), P]
        L.orc_preint_reintegrate.argtypes = [C.POINTER(Preint), C.POINTER(ImuParams), P, C.POINTER(State), P]
        L.orc_preint_free.argtypes = [C.POINTER(Preint)]
        L.orc_preint_factor_eval.argtypes = [C.POINTER(Preint), C.POINTER(C.c_void_p), P,
                                             C.POINTER(C.c_void_p)]
        L.orc_earth_iewn.argtypes = [P, P, P]
        L.orc_reproj_eval.argtypes = [C.POINTER(ReprojConst), C.POINTER(C.c_void_p), P, C.POINTER(C.c_void_p)]
        L.orc_pose_plus.argtypes = [P, P, P]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


# ------------------------------------------------------------------ KLT
def build_pyramid(img: np.ndarray, max_level=3, win=21):
    """-> list of unpadded levels (u8 arrays)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    pyr = Pyramid()
    lib().orc_build_pyramid(_p(img), w, h, w, win, max_level, C.byref(pyr))
    out = []
    for l in range(pyr.nlevels):
        pl = pyr.lv[l]
        buf = np.ctypeslib.as_array(pl.buf, shape=((pl.h + 2 * pl.pad) * pl.pitch,))
        a = buf.reshape(pl.h + 2 * pl.pad, pl.pitch)[pl.pad:pl.pad + pl.h, pl.pad:pl.pad + pl.w].copy()
        out.append(a)
    lib().orc_free_pyramid(C.byref(pyr))
    return out


def scharr(level: np.ndarray) -> np.ndarray:
    """calcSharrDeriv of an image -> int16 [h, w, 2] (dx, dy)."""
    level = np.ascontiguousarray(level, np.uint8)
    h, w = level.shape
    pad = 2
    buf = np.pad(level, pad, mode="reflect")  # numpy 'reflect' == REFLECT_101
    buf = np.ascontiguousarray(buf)
    pl = U8Plane(w, h, pad, w + 2 * pad, buf.ctypes.data_as(C.POINTER(C.c_uint8)))
    out = np.zeros((h, w, 2), np.int16)
    lib().orc_scharr(C.byref(pl), _p(out))
    return out


def calc_optical_flow_pyr_lk(prev, nxt, prev_pts, next_pts=None, params=None, nthreads=1):
    p = params or KltParams.default()
    prev = np.ascontiguousarray(prev, np.uint8)
    nxt = np.ascontiguousarray(nxt, np.uint8)
    h, w = prev.shape
    pp = np.ascontiguousarray(prev_pts, np.float32).reshape(-1, 2)
    n = pp.shape[0]
    npts = pp.copy() if next_pts is None else np.ascontiguousarray(next_pts, np.float32).reshape(-1, 2).copy()
    st = np.zeros(n, np.uint8)
    err = np.zeros(n, np.float32)
    lib().orc_calc_optical_flow_pyr_lk(_p(prev), _p(nxt), w, h, w, _p(pp), _p(npts), _p(st), _p(err), n,
                                       C.byref(p), nthreads)
    return npts, st, err


def klt_fb(prev, nxt, prev_pts, init_pts, cam_w=None, cam_h=None, fb=0.5, border=5.0, params=None,
           reuse_pyramids=False, nthreads=1):
    p = params or KltParams.default()
    prev = np.ascontiguousarray(prev, np.uint8)
    nxt = np.ascontiguousarray(nxt, np.uint8)
    h, w = prev.shape
    pp = np.ascontiguousarray(prev_pts, np.float32).reshape(-1, 2)
    n = pp.shape[0]
    nx = np.ascontiguousarray(init_pts, np.float32).reshape(-1, 2).copy()
    back = np.zeros_like(pp)
    stf = np.zeros(n, np.uint8)
    stb = np.zeros(n, np.uint8)
    keep = np.zeros(n, np.uint8)
    kept = np.zeros(max(n, 1), np.int32)
    k = lib().orc_klt_fb(_p(prev), _p(nxt), w, h, w, _p(pp), _p(nx), _p(back), _p(stf), _p(stb), _p(keep),
                         _p(kept), n, fb, border, cam_w or w, cam_h or h, C.byref(p),
                         1 if reuse_pyramids else 0, nthreads)
    return dict(next=nx, back=back, st_f=stf, st_b=stb, keep=keep, kept_idx=kept[:k].copy())
