"""gvx -- Python host mirror of the MI355X-native IC-GVINS front end.

Thin ctypes layer over libgvx.so (C ABI: include/gvx.h).  The product path is
the HIP library; there is no CPU fallback: importing works anywhere, but every
compute call goes through libgvx.so and raises GvxError if the library or a
gfx950 device is missing.

Interfaces mirror the reference call sites (paths relative to
/root/reference/ic_gvins/ic_gvins/):
  Context.calc_optical_flow_pyr_lk  cv::calcOpticalFlowPyrLK at tracking/tracking.cc:385
  Context.track_fb                  tracking/tracking.cc:380-408 (fwd+bwd+FB+reduceVector)
  Context.klt_fb_batch              the batched frame-pair unit
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgvx.so")

GVX_OK = 0
GVX_PREINT_NORMAL = 0
GVX_PREINT_EARTH = 2


class GvxError(RuntimeError):
    pass


class KltParams(C.Structure):
    _fields_ = [("win", C.c_int32), ("max_level", C.c_int32), ("max_iter", C.c_int32),
                ("eps", C.c_double), ("use_initial_flow", C.c_int32), ("min_eig", C.c_float)]

    @classmethod
    def default(cls, **kw) -> "KltParams":
        p = cls(21, 3, 30, 0.01, 1, 1e-4)
        for k, v in kw.items():
            setattr(p, k, v)
        return p


_lib = None


def lib():
    """Load libgvx.so (raises GvxError when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise GvxError(f"{LIB_PATH} not built: run __graft_entry__.build() or make -C ic-gvins_amd/csrc")
        _lib = C.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


def _declare(L):
    P = C.c_void_p
    i32, i64, f64, u64 = C.c_int32, C.c_int64, C.c_double, C.c_uint64
    sig = {
        "gvx_create": (i32, [i32, C.POINTER(P)]),
        "gvx_destroy": (None, [P]),
        "gvx_status_string": (C.c_char_p, [i32]),
        "gvx_last_error": (C.c_char_p, [P]),
        "gvx_sync": (i32, [P]),
        "gvx_get_stream": (P, [P]),
        "gvx_version": (C.c_char_p, []),
        "gvx_profile_enable": (i32, [P, i32]),
        "gvx_profile_read": (i32, [P, C.c_char_p, C.POINTER(f64), C.POINTER(i64)]),
        "gvx_profile_reset": (i32, [P]),
        "gvx_klt_params_default": (None, [C.POINTER(KltParams)]),
        "gvx_frame_put": (i32, [P, u64, P, i32, i32, i32, C.POINTER(KltParams)]),
        "gvx_frame_drop": (i32, [P, u64]),
        "gvx_frame_level": (i32, [P, u64, i32, P, C.POINTER(i32), C.POINTER(i32)]),
        "gvx_klt": (i32, [P, u64, u64, P, P, P, P, i32, C.POINTER(KltParams)]),
        "gvx_klt_fb": (i32, [P, u64, u64, P, P, P, P, P, P, P, P, i32, f64, f64, i32, i32,
                             C.POINTER(KltParams)]),
        "gvx_klt_fb_batch_dev": (i32, [P, i32, i32, i32, P, P, i32, P, P, P, P, P, P, f64, f64, i32,
                                       i32, C.POINTER(KltParams)]),
        "gvx_klt_fb_batch": (i32, [P, i32, i32, i32, P, P, i32, P, P, P, P, P, P, f64, f64, i32, i32,
                                   C.POINTER(KltParams)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _f32xy(a) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a.reshape(-1, 2)


class Context:
    """One gvx_ctx (device memory, HIP stream, frame-pyramid cache)."""

    def __init__(self, device: int = 0):
        L = lib()
        h = C.c_void_p()
        s = L.gvx_create(device, C.byref(h))
        if s != GVX_OK:
            raise GvxError(f"gvx_create({device}) failed: {L.gvx_status_string(s).decode()}")
        self._h = h
        self._L = L

    def close(self):
        if getattr(self, "_h", None):
            self._L.gvx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    def _check(self, s: int, what: str):
        if s != GVX_OK:
            msg = self._L.gvx_last_error(self._h).decode()
            raise GvxError(f"{what}: {self._L.gvx_status_string(s).decode()} ({msg})")

    # ---------------------------------------------------------------- misc
    def sync(self):
        self._check(self._L.gvx_sync(self._h), "gvx_sync")

    def stream(self) -> int:
        return self._L.gvx_get_stream(self._h) or 0

    def profile(self, on: bool):
        self._check(self._L.gvx_profile_enable(self._h, 1 if on else 0), "profile_enable")

    def profile_reset(self):
        self._check(self._L.gvx_profile_reset(self._h), "profile_reset")

    def profile_read(self, family: str):
        ms, n = C.c_double(), C.c_int64()
        self._check(self._L.gvx_profile_read(self._h, family.encode(), C.byref(ms), C.byref(n)),
                    "profile_read")
        return ms.value, n.value

    # --------------------------------------------------------------- frames
    def frame_put(self, fid: int, gray: np.ndarray, params: Optional[KltParams] = None):
        g = np.ascontiguousarray(gray, dtype=np.uint8)
        if g.ndim != 2:
            raise ValueError("gray image must be 2-D u8")
        p = params or KltParams.default()
        h, w = g.shape
        self._check(self._L.gvx_frame_put(self._h, fid, _ptr(g), w, h, w, C.byref(p)), "frame_put")

    def frame_drop(self, fid: int):
        self._check(self._L.gvx_frame_drop(self._h, fid), "frame_drop")

    def frame_level(self, fid: int, level: int) -> np.ndarray:
        w, h = C.c_int32(), C.c_int32()
        self._check(self._L.gvx_frame_level(self._h, fid, level, None, C.byref(w), C.byref(h)),
                    "frame_level")
        out = np.empty((h.value, w.value), np.uint8)
        self._check(self._L.gvx_frame_level(self._h, fid, level, _ptr(out), None, None), "frame_level")
        return out

    # ------------------------------------------------------------------ KLT
    def calc_optical_flow_pyr_lk(self, prev_id: int, next_id: int, prev_pts, next_pts=None,
                                 params: Optional[KltParams] = None):
        """cv::calcOpticalFlowPyrLK on cached frames -> (next_pts, status, err)."""
        p = params or KltParams.default()
        prev = _f32xy(prev_pts)
        n = prev.shape[0]
        nxt = prev.copy() if next_pts is None else _f32xy(next_pts).copy()
        st = np.zeros(n, np.uint8)
        err = np.zeros(n, np.float32)
        self._check(self._L.gvx_klt(self._h, prev_id, next_id, _ptr(prev), _ptr(nxt), _ptr(st),
                                    _ptr(err), n, C.byref(p)), "gvx_klt")
        return nxt, st, err

    def track_fb(self, prev_id: int, next_id: int, prev_pts, init_pts, cam_w: int, cam_h: int,
                 fb_thresh: float = 0.5, border: float = 5.0, params: Optional[KltParams] = None):
        """tracking.cc:380-408 -> dict(next, back, st_f, st_b, keep, kept_idx)."""
        p = params or KltParams.default()
        prev = _f32xy(prev_pts)
        n = prev.shape[0]
        nxt = _f32xy(init_pts).copy()
        back = np.zeros_like(prev)
        stf = np.zeros(n, np.uint8)
        stb = np.zeros(n, np.uint8)
        keep = np.zeros(n, np.uint8)
        kept = np.zeros(max(n, 1), np.int32)
        nk = C.c_int32()
        self._check(self._L.gvx_klt_fb(self._h, prev_id, next_id, _ptr(prev), _ptr(nxt), _ptr(back),
                                       _ptr(stf), _ptr(stb), _ptr(keep), _ptr(kept), C.byref(nk), n,
                                       fb_thresh, border, cam_w, cam_h, C.byref(p)), "gvx_klt_fb")
        return dict(next=nxt, back=back, st_f=stf, st_b=stb, keep=keep, kept_idx=kept[:nk.value].copy())

    def klt_fb_batch(self, prev_imgs, next_imgs, prev_pts, init_pts, cam_w=None, cam_h=None,
                     fb_thresh: float = 0.5, border: float = 5.0, params: Optional[KltParams] = None):
        """Batched frame-pair unit on host arrays: images [P,H,W] u8, points [P,N,2]."""
        p = params or KltParams.default()
        I = np.ascontiguousarray(prev_imgs, dtype=np.uint8)
        J = np.ascontiguousarray(next_imgs, dtype=np.uint8)
        P, H, W = I.shape
        pp = np.ascontiguousarray(prev_pts, dtype=np.float32).reshape(P, -1, 2)
        N = pp.shape[1]
        nxt = np.ascontiguousarray(init_pts, dtype=np.float32).reshape(P, N, 2).copy()
        back = np.zeros_like(nxt)
        flags = np.zeros((P, N), np.uint8)
        kept = np.zeros((P, max(N, 1)), np.int32)
        nk = np.zeros(P, np.int32)
        self._check(self._L.gvx_klt_fb_batch(self._h, P, W, H, _ptr(I), _ptr(J), N, _ptr(pp), _ptr(nxt),
                                             _ptr(back), _ptr(flags), _ptr(kept), _ptr(nk), fb_thresh,
                                             border, cam_w or W, cam_h or H, C.byref(p)),
                    "gvx_klt_fb_batch")
        return dict(next=nxt, back=back, flags=flags, kept=kept, n_kept=nk)

    def klt_fb_batch_dev(self, n_pairs, w, h, d_prev, d_next, n_pts, d_prev_xy, d_next_xy, d_back_xy,
                         d_flags, d_kept, d_nkept, cam_w=None, cam_h=None, fb_thresh=0.5, border=5.0,
                         params: Optional[KltParams] = None):
        """Device-pointer batch (pointers as ints), enqueued on this context's stream."""
        p = params or KltParams.default()
        self._check(self._L.gvx_klt_fb_batch_dev(self._h, n_pairs, w, h, d_prev, d_next, n_pts,
                                                 d_prev_xy, d_next_xy, d_back_xy, d_flags, d_kept,
                                                 d_nkept, fb_thresh, border, cam_w or w, cam_h or h,
                                                 C.byref(p)), "gvx_klt_fb_batch_dev")
