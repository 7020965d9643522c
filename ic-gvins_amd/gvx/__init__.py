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
LIB_PATH = os.environ.get("GVX_LIB") or os.path.join(_HERE, "libgvx.so")  # GVX_LIB: A/B builds (tools/variant.sh)

GVX_OK = 0
GVX_ERR_NUMERIC = -7  # include/gvx.h: a factorisation met a non-positive pivot
GVX_PREINT_NORMAL = 0
GVX_PREINT_EARTH = 2


class GvxError(RuntimeError):
    pass


# gvx_set_marg_solver (include/gvx.h GVX_MARG_SOLVER_*)
MARG_SOLVER_EXACT, MARG_SOLVER_FAST = 0, 1
# gvx_set_preint_path (include/gvx.h GVX_PREINT_PATH_*)
PREINT_PATH_AUTO, PREINT_PATH_ONEPHASE = 0, 1

# gvx_klt_params.accum (include/gvx.h GVX_LK_ACCUM_*): LK's window-sum order
LK_ACCUM_EXACT, LK_ACCUM_F32_SCALAR, LK_ACCUM_F32_SIMD4 = 0, 1, 2


class KltParams(C.Structure):
    _fields_ = [("win", C.c_int32), ("max_level", C.c_int32), ("max_iter", C.c_int32),
                ("eps", C.c_double), ("use_initial_flow", C.c_int32), ("min_eig", C.c_float),
                ("accum", C.c_int32)]

    @classmethod
    def default(cls, **kw) -> "KltParams":
        p = cls(21, 3, 30, 0.01, 1, 1e-4, LK_ACCUM_EXACT)
        for k, v in kw.items():
            setattr(p, k, v)
        return p


IMU_DTYPE = np.dtype([("time", "f8"), ("dt", "f8"), ("dtheta", "f8", 3), ("dvel", "f8", 3),
                      ("odovel", "f8")], align=True)
STATE_DTYPE = np.dtype([("time", "f8"), ("p", "f8", 3), ("q", "f8", 4), ("v", "f8", 3), ("bg", "f8", 3),
                        ("ba", "f8", 3)], align=True)
PREINT_DTYPE = np.dtype([("variant", "i4"), ("m", "i4"), ("delta_time", "f8"), ("start_time", "f8"),
                         ("end_time", "f8"), ("current", STATE_DTYPE), ("delta", STATE_DTYPE),
                         ("gravity", "f8", 3), ("iewn", "f8", 3), ("q0", "f8", 4),
                         ("jacobian", "f8", 225), ("covariance", "f8", 225),
                         ("sqrt_info", "f8", 225)], align=True)
REPROJ_DTYPE = np.dtype([("pts0", "f8", 3), ("pts1", "f8", 3), ("vel0", "f8", 3), ("vel1", "f8", 3),
                         ("td0", "f8"), ("td1", "f8"), ("std", "f8")], align=True)


class ImuParams(C.Structure):
    _fields_ = [(k, C.c_double) for k in ("acc_vrw", "gyr_arw", "gyr_bias_std", "acc_bias_std",
                                           "corr_time", "gravity")]


class DetectParams(C.Structure):
    _fields_ = [("block_size", C.c_double), ("max_features", C.c_int32), ("quality", C.c_double),
                ("subpix_win", C.c_int32), ("subpix_iters", C.c_int32), ("subpix_eps", C.c_double)]

    @classmethod
    def default(cls, **kw) -> "DetectParams":
        p = cls(200.0, 150, 0.01, 5, 20, 0.01)
        for k, v in kw.items():
            setattr(p, k, v)
        return p


class ClaheParams(C.Structure):
    """cv::createCLAHE(clipLimit, tileGridSize) -- tracking.cc:63 uses (3.0, (21, 21))."""
    _fields_ = [("clip_limit", C.c_double), ("tiles_x", C.c_int32), ("tiles_y", C.c_int32),
                ("channels", C.c_int32)]

    @classmethod
    def default(cls, **kw) -> "ClaheParams":
        p = cls(3.0, 21, 21, 1)
        for k, v in kw.items():
            setattr(p, k, v)
        return p


def _frame_and_params(img, params):
    """A MONO8 (h x w) or BGR8 (h x w x 3) frame and CLAHE params whose channels
    field says which (gvx_clahe_params.channels)."""
    g = np.ascontiguousarray(img, dtype=np.uint8)
    if g.ndim == 3 and g.shape[2] == 3:
        ch = 3
    elif g.ndim == 2:
        ch = 1
    else:
        raise ValueError("frame must be h x w (MONO8) or h x w x 3 (BGR8) u8")
    p = params or ClaheParams.default()
    p = ClaheParams(p.clip_limit, p.tiles_x, p.tiles_y, ch)
    return g, p


class Camera(C.Structure):
    """gvx_camera: Camera (tracking/camera.cc:25-46), K = [fx skew cx; 0 fy cy; 0 0 1],
    distortion (k1, k2, p1, p2, k3)."""
    _fields_ = [(k, C.c_double) for k in ("fx", "fy", "cx", "cy", "skew", "k1", "k2", "p1", "p2", "k3")] + \
               [("width", C.c_int32), ("height", C.c_int32)]


class InsConfig(C.Structure):
    """gvx_ins_config: IntegrationConfiguration as insMechanization reads it
    (integration_state.h:91-99)."""
    _fields_ = [("iswithearth", C.c_int32), ("gravity", C.c_double * 3), ("iewn", C.c_double * 3)]

    @classmethod
    def make(cls, iswithearth, gravity, iewn=(0.0, 0.0, 0.0)) -> "InsConfig":
        c = cls()
        c.iswithearth = 1 if iswithearth else 0
        for i in range(3):
            c.gravity[i] = float(gravity[i])
            c.iewn[i] = float(iewn[i])
        return c


# GVX_FACTOR_* kind -> (residuals, parameter block size, constants per factor)
SMALL_FACTOR_DIMS = {0: (3, 7, 9), 1: (6, 9, 0), 2: (6, 7, 13), 3: (9, 9, 18)}
FACTOR_GNSS, FACTOR_IMU_ERROR, FACTOR_POSE_PRIOR, FACTOR_MIX_PRIOR = 0, 1, 2, 3

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
        "gvx_frame_put_dev": (i32, [P, u64, P, i32, i32, i32, P]),
        "gvx_frame_level_padded": (i32, [P, u64, i32, i32, P]),
        "gvx_pyramid_layout": (i32, [i32, i32, i32, P, P, P, P, P, P]),
        "gvx_build_pyramids_dev": (i32, [P, i32, i32, i32, P, i64, i32, i32, P]),
        "gvx_klt": (i32, [P, u64, u64, P, P, P, P, i32, C.POINTER(KltParams)]),
        "gvx_klt_fb": (i32, [P, u64, u64, P, P, P, P, P, P, P, P, i32, f64, f64, i32, i32,
                             C.POINTER(KltParams)]),
        "gvx_klt_fb_batch_dev": (i32, [P, i32, i32, i32, P, P, i32, P, P, P, P, P, P, f64, f64, i32,
                                       i32, C.POINTER(KltParams)]),
        "gvx_klt_fb_batch_init_dev": (i32, [P, i32, i32, i32, P, P, i32, P, P, P, P, P, P, P, f64, f64, i32,
                                            i32, C.POINTER(KltParams)]),
        "gvx_klt_fb_batch": (i32, [P, i32, i32, i32, P, P, i32, P, P, P, P, P, P, f64, f64, i32, i32,
                                   C.POINTER(KltParams)]),
        "gvx_klt_batch_pyramids_dev": (i32, [P, i32, i32, i32, P, P, i32, P]),
        "gvx_klt_fb_batch_pyr_dev": (i32, [P, i32, i32, i32, P, P, P, i32, P, P, P, P, P, P, P, f64, f64, i32,
                                           i32, C.POINTER(KltParams)]),
        "gvx_preint_integrate": (i32, [P, i32, C.POINTER(ImuParams), i32, P, P, P, P, P, P]),
        "gvx_preint_integrate_dev": (i32, [P, i32, C.POINTER(ImuParams), i32, P, P, P, P, P, P]),
        "gvx_earth_iewn": (None, [P, P, P]),
        "gvx_preint_sqrt_info": (i32, [P, i32, P]),
        "gvx_preint_factor_eval": (i32, [P, i32, P, P, i32, P, P, i32, P, P, P]),
        "gvx_preint_factor_eval_dev": (i32, [P, i32, P, P, P, P, P, P, P]),
        "gvx_reproj_eval": (i32, [P, i32, P, P, i32, P, P, P]),
        "gvx_factor_set_create": (i32, [P, i32, P, P, i32, P, P, i32, P, P, i32, P, P, P]),
        "gvx_factor_set_destroy": (None, [P]),
        "gvx_factors_prepare": (i32, [P, i32]),
        "gvx_factor_read_reproj": (i32, [P, i32, P, P]),
        "gvx_factor_read_preint": (i32, [P, i32, P, P]),
        "gvx_reproj_eval_dev": (i32, [P, i32, P, P, P, P, P]),
        "gvx_factor_batch_eval_dev": (i32, [P, i32, P, P, P, P, i32, P, P, P, P, P, P, P]),
        "gvx_detect_params_default": (None, [C.POINTER(DetectParams)]),
        "gvx_detect": (i32, [P, u64, P, i32, P, i32, i32, i32, C.POINTER(DetectParams), P, P, C.POINTER(i32)]),
        "gvx_clahe_params_default": (None, [C.POINTER(ClaheParams)]),
        "gvx_undistort_points": (i32, [P, C.POINTER(Camera), i32, P, P]),
        "gvx_undistort_points_dev": (i32, [P, C.POINTER(Camera), i32, P, P]),
        "gvx_distort_points": (i32, [P, C.POINTER(Camera), i32, P, P]),
        "gvx_distort_points_dev": (i32, [P, C.POINTER(Camera), i32, P, P]),
        "gvx_predict_rotated": (i32, [P, C.POINTER(Camera), P, i32, P, P]),
        "gvx_predict_rotated_dev": (i32, [P, C.POINTER(Camera), P, i32, P, P]),
        "gvx_project_points": (i32, [P, C.POINTER(Camera), P, P, i32, P, P]),
        "gvx_project_points_dev": (i32, [P, C.POINTER(Camera), P, P, i32, P, P]),
        "gvx_point_velocity": (i32, [P, C.POINTER(Camera), i32, P, P, f64, P]),
        "gvx_point_velocity_dev": (i32, [P, C.POINTER(Camera), i32, P, P, f64, P]),
        "gvx_keypoint_parallax": (i32, [P, C.POINTER(Camera), P, P, i32, P, P, P]),
        "gvx_keypoint_parallax_dev": (i32, [P, C.POINTER(Camera), P, P, i32, P, P, P]),
        "gvx_clahe_batch_dev": (i32, [P, i32, i32, i32, P, i64, i32, P, i64, i32, C.POINTER(ClaheParams), P]),
        "gvx_clahe": (i32, [P, i32, i32, P, i32, P, i32, C.POINTER(ClaheParams), P]),
        "gvx_frame_preprocess": (i32, [P, u64, P, i32, i32, i32, C.POINTER(ClaheParams), C.POINTER(KltParams),
                                       P, P]),
        "gvx_frame_preprocess_dev": (i32, [P, u64, P, i32, i32, i32, C.POINTER(ClaheParams),
                                           C.POINTER(KltParams), P, P]),
        "gvx_frame_preprocess_indexed_dev": (i32, [P, u64, P, i64, P, i32, i32, i32, i32, C.POINTER(ClaheParams),
                                                   C.POINTER(KltParams), P]),
        "gvx_ins_propagate": (i32, [P, C.POINTER(InsConfig), i32, P, P, P, P]),
        "gvx_ins_propagate_dev": (i32, [P, C.POINTER(InsConfig), i32, P, P, P, P]),
        "gvx_redo_ins_mechanization": (i32, [P, C.POINTER(InsConfig), P, i32, P, P, C.POINTER(i32)]),
        "gvx_imu_series_from_to": (i32, [P, i32, f64, f64, P, C.POINTER(i32)]),
        "gvx_small_factor_eval": (i32, [P, i32, i32, P, P, i32, P, P, P]),
        "gvx_small_factor_eval_dev": (i32, [P, i32, i32, P, P, P, P, P]),
        "gvx_marg_factor_eval": (i32, [P, i32, i32, P, P, P, i32, P, P, P, P, P, P]),
        "gvx_marginalize": (i32, [P, i32, P, P, P, P, P, P, i64, P, i32, P, P, i32, i32, P, P, P, P, P, P]),
        "gvx_marginalize_dev": (i32, [P, i32, P, P, P, P, P, P, i64, P, i32, P, P, i32, i32, P, P, P, P, P, P]),
        "gvx_schur_solve": (i32, [P, i32, P, P, P, P, P, P, i64, i32, P, P, i32, i32, P, P, P, P]),
        "gvx_schur_solve_dev": (i32, [P, i32, P, P, P, P, P, P, i64, i32, P, P, i32, i32, P, P, P, P]),
        "gvx_sym_eigen": (i32, [P, i32, P, i32, P, P, C.POINTER(i32)]),
        "gvx_set_marg_solver": (i32, [P, i32]),
        "gvx_set_preint_path": (i32, [P, i32]),
        "gvx_set_klt_phases": (i32, [P, i32, i32]),
        "gvx_find_fundamental_ransac": (i32, [P, i32, P, P, P, f64, f64, i32, P, P, P]),
        "gvx_copy_indexed_dev": (i32, [P, P, P, C.c_size_t, P, i32]),
        "gvx_track_record_dev": (i32, [P, P, P, i32, P, P, P, i32]),
        "gvx_track_frame_dev": (i32, [P, u64, u64, i32, P, P, P, P, i32, i32, i32, f64, f64, C.POINTER(KltParams),
                                      C.POINTER(DetectParams), P, P, P]),
        "gvx_track_frame_record_dev": (i32, [P, u64, u64, i32, P, P, P, P, i32, i32, i32, f64, f64,
                                             C.POINTER(KltParams), C.POINTER(DetectParams), P, P, P, i32]),
        "gvx_find_fundamental_ransac_dev": (i32, [P, i32, P, P, P, f64, f64, i32, P, P, P]),
        "gvx_capture_begin": (i32, [P]),
        "gvx_capture_end": (i32, [P, C.POINTER(P)]),
        "gvx_capture_abort": (i32, [P]),
        "gvx_graph_launch": (i32, [P, P]),
        "gvx_graph_destroy": (None, [P]),
        "gvx_copy_dev": (i32, [P, P, P, C.c_size_t]),
        "gvx_branch_begin": (i32, [P]),
        "gvx_branch_end": (i32, [P]),
        "gvx_branch_join": (i32, [P]),
        "gvx_index_advance_dev": (i32, [P, P, i32]),
        "gvx_frame_eig_dev": (i32, [P, u64, P]),
    }
    for name, (res, args) in sig.items():
        # an older build (a GVX_LIB variant timed against the tree) may lack newer
        # entry points: those stay undeclared and fail at their call
        # (tests/test_abi.py holds the in-tree library to every declared symbol)
        fn = getattr(L, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args


def pyramid_layout(w: int, h: int, max_level: int = 3):
    """gvx_pyramid_layout (host only) -> dict(nlev, off, pitch, w, h, bytes) of one
    image pyramid as gvx_build_pyramids_dev writes it."""
    n = C.c_int32()
    off = np.zeros(8, np.int64)
    pitch, lw, lh = (np.zeros(8, np.int32) for _ in range(3))
    b = C.c_int64()
    st = lib().gvx_pyramid_layout(w, h, max_level, C.byref(n), off.ctypes.data, pitch.ctypes.data,
                                  lw.ctypes.data, lh.ctypes.data, C.byref(b))
    if st:
        raise GvxError(f"gvx_pyramid_layout({w}, {h}, {max_level}): status {st}")
    k = n.value
    return dict(nlev=k, off=off[:k], pitch=pitch[:k], w=lw[:k], h=lh[:k], bytes=b.value)


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

    def frame_put_dev(self, fid: int, d_gray: int, w: int, h: int, stride: Optional[int] = None,
                      params: Optional[KltParams] = None):
        """Pyramid of a device-resident image (pointer as int), enqueued without waiting."""
        p = params or KltParams.default()
        self._check(self._L.gvx_frame_put_dev(self._h, fid, d_gray, w, h, stride or w, C.byref(p)),
                    "frame_put_dev")

    # -------------------------------------------------------- preprocessing
    def clahe(self, gray: np.ndarray, params: Optional[ClaheParams] = None, hist_mean: bool = False):
        """clahe_->apply(image, image) (tracking.cc:139); with hist_mean also
        calculateHistigram of the input (tracking.cc:88-105) -> (image, mean).
        An h x w x 3 input is BGR8: converted to gray first (tracking.cc:111-113)."""
        g, p = _frame_and_params(gray, params)
        h, w = g.shape[:2]
        out = np.empty((h, w), np.uint8)
        m = C.c_double()
        self._check(self._L.gvx_clahe(self._h, w, h, _ptr(g), w * p.channels, _ptr(out), w, C.byref(p),
                                      C.byref(m) if hist_mean else None), "clahe")
        return (out, m.value) if hist_mean else out

    def clahe_batch_dev(self, n, w, h, d_src, d_dst, params: Optional[ClaheParams] = None, d_hist_mean=None,
                        src_img_stride=None, src_stride=None, dst_img_stride=None, dst_stride=None):
        self._check(self._L.gvx_clahe_batch_dev(self._h, n, w, h, d_src, src_img_stride or w * h, src_stride or w,
                                                d_dst, dst_img_stride or w * h, dst_stride or w,
                                                C.byref(params or ClaheParams.default()), d_hist_mean),
                    "clahe_batch_dev")

    def frame_preprocess(self, fid: int, gray: np.ndarray, clahe: Optional[ClaheParams] = None,
                         params: Optional[KltParams] = None, hist_mean: bool = False):
        """Tracking::preprocessing (tracking.cc:107-141) into the frame cache:
        -> (equalised image, histogram mean or None).  An h x w x 3 input is BGR8."""
        g, cp = _frame_and_params(gray, clahe)
        h, w = g.shape[:2]
        out = np.empty((h, w), np.uint8)
        m = C.c_double()
        self._check(self._L.gvx_frame_preprocess(self._h, fid, _ptr(g), w, h, w * cp.channels, C.byref(cp),
                                                 C.byref(params or KltParams.default()),
                                                 C.byref(m) if hist_mean else None, _ptr(out)), "frame_preprocess")
        return out, (m.value if hist_mean else None)

    def frame_preprocess_dev(self, fid: int, d_gray: int, w: int, h: int, stride: Optional[int] = None,
                             clahe: Optional[ClaheParams] = None, params: Optional[KltParams] = None,
                             d_hist_mean=None, d_clahe_out=None):
        self._check(self._L.gvx_frame_preprocess_dev(self._h, fid, d_gray, w, h, stride or w,
                                                     C.byref(clahe or ClaheParams.default()),
                                                     C.byref(params or KltParams.default()), d_hist_mean,
                                                     d_clahe_out), "frame_preprocess_dev")

    def frame_preprocess_indexed_dev(self, fid: int, d_frames: int, frame_stride: int, d_index: int, n_frames: int,
                                     w: int, h: int, stride: Optional[int] = None, clahe: Optional[ClaheParams] = None,
                                     params: Optional[KltParams] = None, d_hist_mean=None):
        """Preprocess frame *d_index (clamped to [0, n_frames - 1]) of an HBM-resident
        sequence (index read on the device)."""
        self._check(self._L.gvx_frame_preprocess_indexed_dev(self._h, fid, d_frames, frame_stride, d_index,
                                                             n_frames, w, h,
                                                             stride or w, C.byref(clahe or ClaheParams.default()),
                                                             C.byref(params or KltParams.default()), d_hist_mean),
                    "frame_preprocess_indexed_dev")

    # ----------------------------------------------------------- camera ops
    def track_frame_dev(self, prev_id: int, next_id: int, track: bool, d_pts, d_vel, d_init, d_n, capacity: int,
                        cam_w: int, cam_h: int, klt: Optional[KltParams] = None,
                        detect: Optional[DetectParams] = None, fb_thresh=0.5, border=5.0, d_kept=None,
                        d_corners=None, d_n_corners=None):
        """One frame of Tracking::track's image path with the tracker state in
        device memory (pointers as ints), no host round trip (gvx_track_frame_dev)."""
        kp = klt or KltParams.default()
        dp = detect or DetectParams.default()
        self._check(self._L.gvx_track_frame_dev(self._h, prev_id, next_id, 1 if track else 0, d_pts, d_vel, d_init,
                                                d_n, capacity, cam_w, cam_h, fb_thresh, border, C.byref(kp),
                                                C.byref(dp), d_kept, d_corners, d_n_corners),
                    "gvx_track_frame_dev")

    def track_frame_record_dev(self, prev_id: int, next_id: int, track: bool, d_pts, d_vel, d_init, d_n,
                               capacity: int, cam_w: int, cam_h: int, d_tracks, d_counts, d_frame_index,
                               max_frames: int, klt: Optional[KltParams] = None,
                               detect: Optional[DetectParams] = None, fb_thresh=0.5, border=5.0):
        """track_frame_dev then track_record_dev, the record fused into the last kernel."""
        kp = klt or KltParams.default()
        dp = detect or DetectParams.default()
        self._check(self._L.gvx_track_frame_record_dev(self._h, prev_id, next_id, 1 if track else 0, d_pts, d_vel,
                                                       d_init, d_n, capacity, cam_w, cam_h, fb_thresh, border,
                                                       C.byref(kp), C.byref(dp), d_tracks, d_counts, d_frame_index,
                                                       max_frames), "gvx_track_frame_record_dev")

    def frame_eig_dev(self, frame_id: int, detect: Optional[DetectParams] = None):
        """The detection's eigenvalue map of a cached frame, kept with the frame for
        the next tracking call on it (gvx_frame_eig_dev)."""
        dp = detect or DetectParams.default()
        self._check(self._L.gvx_frame_eig_dev(self._h, frame_id, C.byref(dp)), "gvx_frame_eig_dev")

    def copy_indexed_dev(self, d_dst: int, d_src_base: int, nbytes: int, d_index: int, n_src: int):
        self._check(self._L.gvx_copy_indexed_dev(self._h, d_dst, d_src_base, nbytes, d_index, n_src),
                    "gvx_copy_indexed_dev")

    def track_record_dev(self, d_pts: int, d_n: int, capacity: int, d_tracks: int, d_counts: int,
                         d_frame_index: int, max_frames: int):
        self._check(self._L.gvx_track_record_dev(self._h, d_pts, d_n, capacity, d_tracks, d_counts, d_frame_index,
                                                 max_frames), "gvx_track_record_dev")

    def index_advance_dev(self, d_index: int, delta: int = 1):
        """*d_index += delta on the context stream (gvx_index_advance_dev)."""
        self._check(self._L.gvx_index_advance_dev(self._h, d_index, delta), "gvx_index_advance_dev")

    def find_fundamental_ransac(self, sets, thresh=1.5, confidence=0.99, max_iters=1000):
        """cv::findFundamentalMat(p1, p2, FM_RANSAC, thresh, confidence, mask) per
        (p1, p2) pair of float [n, 2] arrays in `sets` (tracking.cc:547-548) ->
        list of (result, mask u8 [n], F [3, 3])."""
        n = [len(np.asarray(a).reshape(-1, 2)) for a, _ in sets]
        off = np.zeros(len(sets) + 1, np.int32)
        off[1:] = np.cumsum(n)
        p1 = np.ascontiguousarray(np.concatenate([np.asarray(a, np.float32).reshape(-1, 2) for a, _ in sets]))
        p2 = np.ascontiguousarray(np.concatenate([np.asarray(b, np.float32).reshape(-1, 2) for _, b in sets]))
        mask = np.zeros(max(int(off[-1]), 1), np.uint8)
        F = np.zeros((len(sets), 9))
        res = np.zeros(len(sets), np.int32)
        self._check(self._L.gvx_find_fundamental_ransac(self._h, len(sets), _ptr(off), _ptr(p1), _ptr(p2), thresh,
                                                        confidence, max_iters, _ptr(mask), _ptr(F), _ptr(res)),
                    "gvx_find_fundamental_ransac")
        return [(int(res[i]), mask[off[i]:off[i + 1]].copy(), F[i].reshape(3, 3)) for i in range(len(sets))]

    def find_fundamental_ransac_dev(self, n_sets, d_off, d_p1, d_p2, d_mask, d_F, d_result, thresh=1.5,
                                    confidence=0.99, max_iters=1000):
        self._check(self._L.gvx_find_fundamental_ransac_dev(self._h, n_sets, d_off, d_p1, d_p2, thresh, confidence,
                                                            max_iters, d_mask, d_F, d_result),
                    "gvx_find_fundamental_ransac_dev")

    def undistort_points(self, cam: Camera, pts):
        """Camera::undistortPoints (camera.cc:72-74)."""
        p = _f32xy(pts)
        out = np.empty_like(p)
        self._check(self._L.gvx_undistort_points(self._h, C.byref(cam), len(p), _ptr(p), _ptr(out)), "undistort")
        return out

    def distort_points(self, cam: Camera, pts):
        """Camera::distortPoints (camera.cc:76-89)."""
        p = _f32xy(pts)
        out = np.empty_like(p)
        self._check(self._L.gvx_distort_points(self._h, C.byref(cam), len(p), _ptr(p), _ptr(out)), "distort")
        return out

    def predict_rotated(self, cam: Camera, r_cur_pre, pts):
        """trackReferenceFrame's rotation-compensated initial flow (tracking.cc:465-478)."""
        p = _f32xy(pts)
        R = np.ascontiguousarray(r_cur_pre, np.float64).reshape(9)
        out = np.empty_like(p)
        self._check(self._L.gvx_predict_rotated(self._h, C.byref(cam), _ptr(R), len(p), _ptr(p), _ptr(out)),
                    "predict_rotated")
        return out

    def project_points(self, cam: Camera, R, t, pw):
        """trackMappoint's prediction: world2pixel + distortPoints (tracking.cc:366-377)."""
        R = np.ascontiguousarray(R, np.float64).reshape(9)
        t = np.ascontiguousarray(t, np.float64).reshape(3)
        pw = np.ascontiguousarray(pw, np.float64).reshape(-1, 3)
        out = np.empty((len(pw), 2), np.float32)
        self._check(self._L.gvx_project_points(self._h, C.byref(cam), _ptr(R), _ptr(t), len(pw), _ptr(pw),
                                               _ptr(out)), "project_points")
        return out

    def point_velocity(self, cam: Camera, pre, cur, dt: float):
        """(pixel2cam(cur) - pixel2cam(pre)) / dt (tracking.cc:433, :530)."""
        a, b = _f32xy(pre), _f32xy(cur)
        out = np.empty((len(a), 2), np.float64)
        self._check(self._L.gvx_point_velocity(self._h, C.byref(cam), len(a), _ptr(a), _ptr(b), dt, _ptr(out)),
                    "point_velocity")
        return out

    def keypoint_parallax(self, cam: Camera, R0, R1, ref, cur):
        """Tracking::keyPointParallax (tracking.cc:861-871) per point pair."""
        a, b = _f32xy(ref), _f32xy(cur)
        R0 = np.ascontiguousarray(R0, np.float64).reshape(9)
        R1 = np.ascontiguousarray(R1, np.float64).reshape(9)
        out = np.empty(len(a), np.float64)
        self._check(self._L.gvx_keypoint_parallax(self._h, C.byref(cam), _ptr(R0), _ptr(R1), len(a), _ptr(a),
                                                  _ptr(b), _ptr(out)), "keypoint_parallax")
        return out

    def frame_drop(self, fid: int):
        self._check(self._L.gvx_frame_drop(self._h, fid), "frame_drop")

    def frame_level(self, fid: int, level: int) -> np.ndarray:
        w, h = C.c_int32(), C.c_int32()
        self._check(self._L.gvx_frame_level(self._h, fid, level, None, C.byref(w), C.byref(h)),
                    "frame_level")
        out = np.empty((h.value, w.value), np.uint8)
        self._check(self._L.gvx_frame_level(self._h, fid, level, _ptr(out), None, None), "frame_level")
        return out

    def frame_level_padded(self, fid: int, level: int, pad: int = 32) -> np.ndarray:
        """Level `level` with its REFLECT_101 border of `pad` pixels."""
        w, h = C.c_int32(), C.c_int32()
        self._check(self._L.gvx_frame_level(self._h, fid, level, None, C.byref(w), C.byref(h)),
                    "frame_level")
        out = np.empty((h.value + 2 * pad, w.value + 2 * pad), np.uint8)
        self._check(self._L.gvx_frame_level_padded(self._h, fid, level, pad, _ptr(out)), "frame_level_padded")
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

    # ------------------------------------------------------------ detection
    def detect(self, frame_id: int, count_xy=None, mask_xy=None, ismask: bool = True, n_existing: int = 0,
               params: Optional[DetectParams] = None):
        """Tracking::featuresDetection on a cached frame -> (corners [n,2] f32 or
        None when the early exit triggers, per-block counts)."""
        p = params or DetectParams.default()
        cxy = np.zeros((0, 2), np.float32) if count_xy is None else _f32xy(count_xy)
        mxy = np.zeros((0, 2), np.float32) if mask_xy is None else _f32xy(mask_xy)
        # block_cnts * max_block_features bounds the output
        cap = 4096
        out = np.zeros((cap, 2), np.float32)
        blk = np.zeros(1024, np.int32)
        n = C.c_int32()
        self._check(self._L.gvx_detect(self._h, frame_id, _ptr(cxy), cxy.shape[0], _ptr(mxy), mxy.shape[0],
                                       1 if ismask else 0, n_existing, C.byref(p), _ptr(out), _ptr(blk),
                                       C.byref(n)), "gvx_detect")
        if n.value < 0:
            return None, blk[:0]
        return out[:n.value].copy(), blk

    # ------------------------------------------------------- preintegration
    def preint_integrate(self, variant: int, prm, segments, states, iewn=None):
        """Preintegrate a batch of IMU segments (list of IMU_DTYPE arrays, each the
        vector<IMU> of one time-node interval, ic_gvins.cc:940-953).
        prm: (acc_vrw, gyr_arw, gyr_bias_std, acc_bias_std, corr_time, gravity).
        states: STATE_DTYPE array [n_seg]; iewn: [n_seg, 3] (Earth variant).
        Returns (PREINT_DTYPE results [n_seg], pn [sum(m-1), 4], pn offsets [n_seg])."""
        segs = [np.ascontiguousarray(s, dtype=IMU_DTYPE) for s in segments]
        n = len(segs)
        off = np.zeros(n + 1, np.int32)
        off[1:] = np.cumsum([len(s) for s in segs])
        imu = np.concatenate(segs) if n else np.zeros(0, IMU_DTYPE)
        st = np.ascontiguousarray(states, dtype=STATE_DTYPE).reshape(n)
        iw = None if iewn is None else np.ascontiguousarray(iewn, np.float64).reshape(n, 3)
        out = np.zeros(n, PREINT_DTYPE)
        pn_off = (off[:-1] - np.arange(n)).astype(np.int32)
        pn = np.zeros((max(int(off[-1]) - n, 1), 4))
        p = ImuParams(*prm)
        self._check(self._L.gvx_preint_integrate(self._h, variant, C.byref(p), n, _ptr(imu), _ptr(off), _ptr(st),
                                                 _ptr(iw), _ptr(out), _ptr(pn)), "gvx_preint_integrate")
        return out, pn[:int(off[-1]) - n], pn_off

    def preint_sqrt_info(self, pre):
        """Fill pre[i].sqrt_info = LLT(covariance^-1).matrixL()^T (gvx_preint_sqrt_info)
        for preintegration results formed elsewhere; returns the updated copy."""
        out = np.ascontiguousarray(pre, dtype=PREINT_DTYPE).copy()
        self._check(self._L.gvx_preint_sqrt_info(self._h, out.shape[0], _ptr(out)), "gvx_preint_sqrt_info")
        return out

    def preint_factor_eval(self, pre, pn, pn_off, params, offs, jacobians=True):
        """PreintegrationFactor::Evaluate batch -> (residuals [n,15], jacobians [n,480] or None)."""
        pre = np.ascontiguousarray(pre, dtype=PREINT_DTYPE)
        n = pre.shape[0]
        pn = np.ascontiguousarray(pn, np.float64).reshape(-1, 4)
        pno = np.ascontiguousarray(pn_off, np.int32)
        prm = np.ascontiguousarray(params, np.float64).reshape(-1)
        o = np.ascontiguousarray(offs, np.int32).reshape(n, 4)
        res = np.zeros((n, 15))
        jac = np.zeros((n, 480)) if jacobians else None
        self._check(self._L.gvx_preint_factor_eval(self._h, n, _ptr(pre), _ptr(pn), pn.shape[0], _ptr(pno),
                                                   _ptr(prm), prm.size, _ptr(o), _ptr(res), _ptr(jac)),
                    "gvx_preint_factor_eval")
        return res, jac

    def reproj_eval(self, consts, params, offs, jacobians=True):
        """ReprojectionFactor::Evaluate batch -> (residuals [n,2], jacobians [n,46] or None)."""
        cs = np.ascontiguousarray(consts, dtype=REPROJ_DTYPE)
        n = cs.shape[0]
        prm = np.ascontiguousarray(params, np.float64).reshape(-1)
        o = np.ascontiguousarray(offs, np.int32).reshape(n, 5)
        res = np.zeros((n, 2))
        jac = np.zeros((n, 46)) if jacobians else None
        self._check(self._L.gvx_reproj_eval(self._h, n, _ptr(cs), _ptr(prm), prm.size, _ptr(o), _ptr(res),
                                            _ptr(jac)), "gvx_reproj_eval")
        return res, jac

    def pyramid_layout(self, w: int, h: int, max_level: int = 3):
        return pyramid_layout(w, h, max_level)

    def build_pyramids_dev(self, n_img, w, h, d_imgs, img_stride, stride, max_level, d_out):
        """Device-pointer batched pyramid build (pointers as ints), async on the context stream."""
        self._check(self._L.gvx_build_pyramids_dev(self._h, n_img, w, h, d_imgs, img_stride, stride, max_level,
                                                   d_out), "gvx_build_pyramids_dev")

    def klt_fb_batch_init_dev(self, n_pairs, w, h, d_prev, d_next, n_pts, d_prev_xy, d_init_xy, d_next_xy,
                              d_back_xy, d_flags, d_kept, d_nkept, cam_w=None, cam_h=None, fb_thresh=0.5,
                              border=5.0, params: Optional[KltParams] = None):
        """Device-pointer batch with the initial flow read from d_init_xy (next output only)."""
        p = params or KltParams.default()
        self._check(self._L.gvx_klt_fb_batch_init_dev(self._h, n_pairs, w, h, d_prev, d_next, n_pts, d_prev_xy,
                                                      d_init_xy, d_next_xy, d_back_xy, d_flags, d_kept, d_nkept,
                                                      fb_thresh, border, cam_w or w, cam_h or h, C.byref(p)),
                    "gvx_klt_fb_batch_init_dev")

    def klt_batch_pyramids_dev(self, n_pairs, w, h, d_prev, d_next, max_level, d_pyr):
        """gvx_klt_batch_pyramids_dev: levels >= 1 of the prev then next images of a
        batch into d_pyr (2 * n_pairs * pyramid_layout(w, h, max_level)["bytes"])."""
        self._check(self._L.gvx_klt_batch_pyramids_dev(self._h, n_pairs, w, h, d_prev, d_next, max_level, d_pyr),
                    "gvx_klt_batch_pyramids_dev")

    def klt_fb_batch_pyr_dev(self, n_pairs, w, h, d_prev, d_next, d_pyr, n_pts, d_prev_xy, d_init_xy, d_next_xy,
                             d_back_xy, d_flags, d_kept, d_nkept, cam_w=None, cam_h=None, fb_thresh=0.5,
                             border=5.0, params: Optional[KltParams] = None):
        """klt_fb_batch_init_dev over pyramids built by klt_batch_pyramids_dev."""
        p = params or KltParams.default()
        self._check(self._L.gvx_klt_fb_batch_pyr_dev(self._h, n_pairs, w, h, d_prev, d_next, d_pyr, n_pts,
                                                     d_prev_xy, d_init_xy, d_next_xy, d_back_xy, d_flags, d_kept,
                                                     d_nkept, fb_thresh, border, cam_w or w, cam_h or h,
                                                     C.byref(p)), "gvx_klt_fb_batch_pyr_dev")

    def klt_fb_batch_dev(self, n_pairs, w, h, d_prev, d_next, n_pts, d_prev_xy, d_next_xy, d_back_xy,
                         d_flags, d_kept, d_nkept, cam_w=None, cam_h=None, fb_thresh=0.5, border=5.0,
                         params: Optional[KltParams] = None):
        """Device-pointer batch (pointers as ints), enqueued on this context's stream."""
        p = params or KltParams.default()
        self._check(self._L.gvx_klt_fb_batch_dev(self._h, n_pairs, w, h, d_prev, d_next, n_pts,
                                                 d_prev_xy, d_next_xy, d_back_xy, d_flags, d_kept,
                                                 d_nkept, fb_thresh, border, cam_w or w, cam_h or h,
                                                 C.byref(p)), "gvx_klt_fb_batch_dev")

    def preint_integrate_dev(self, variant, prm, n_seg, d_imu, d_seg_off, d_state0, d_iewn, d_out, d_pn):
        """Device-pointer preintegration batch (pointers as ints), async on the context stream."""
        p = ImuParams(*prm)
        self._check(self._L.gvx_preint_integrate_dev(self._h, variant, C.byref(p), n_seg, d_imu, d_seg_off,
                                                     d_state0, d_iewn, d_out, d_pn), "gvx_preint_integrate_dev")

    def preint_factor_eval_dev(self, n, d_pre, d_pn, d_pn_off, d_params, d_offs, d_res, d_jac):
        """Device-pointer PreintegrationFactor batch, async on the context stream."""
        self._check(self._L.gvx_preint_factor_eval_dev(self._h, n, d_pre, d_pn, d_pn_off, d_params, d_offs,
                                                       d_res, d_jac), "gvx_preint_factor_eval_dev")

    def factor_batch_eval_dev(self, n_r, d_consts, d_roffs, d_rres, d_rjac, n_p, d_pre, d_pn, d_pn_off, d_poffs,
                              d_pres, d_pjac, d_params):
        """Both factor kinds over one parameter array, async on the context stream."""
        self._check(self._L.gvx_factor_batch_eval_dev(self._h, n_r, d_consts, d_roffs, d_rres, d_rjac, n_p, d_pre,
                                                      d_pn, d_pn_off, d_poffs, d_pres, d_pjac, d_params),
                    "gvx_factor_batch_eval_dev")

    def reproj_eval_dev(self, n, d_consts, d_params, d_offs, d_res, d_jac):
        """Device-pointer ReprojectionFactor batch, async on the context stream."""
        self._check(self._L.gvx_reproj_eval_dev(self._h, n, d_consts, d_params, d_offs, d_res, d_jac),
                    "gvx_reproj_eval_dev")

    # ---------------------------------------------- remaining window factors
    def small_factor_eval(self, kind: int, consts, params, offs, jacobians=True):
        """GnssFactor / ImuErrorFactor / ImuPosePriorFactor / ImuMixPriorFactor
        batch (GVX_FACTOR_*) -> (residuals [n, R], jacobians [n, R*P] or None)."""
        if kind not in SMALL_FACTOR_DIMS:
            raise GvxError(f"small_factor_eval: unknown factor kind {kind}")
        R, P, NC = SMALL_FACTOR_DIMS[kind]
        o = np.ascontiguousarray(offs, np.int32).reshape(-1)
        n = o.size
        cs = np.ascontiguousarray(consts, np.float64).reshape(-1) if NC else None
        prm = np.ascontiguousarray(params, np.float64).reshape(-1)
        res = np.zeros((n, R))
        jac = np.zeros((n, R * P)) if jacobians else None
        self._check(self._L.gvx_small_factor_eval(self._h, kind, n, _ptr(cs), _ptr(prm), prm.size, _ptr(o),
                                                  _ptr(res), _ptr(jac)), "gvx_small_factor_eval")
        return res, jac

    def small_factor_eval_dev(self, kind, n, d_consts, d_params, d_offs, d_res, d_jac):
        """Device-pointer small-factor batch, async on the context stream."""
        self._check(self._L.gvx_small_factor_eval_dev(self._h, kind, n, d_consts, d_params, d_offs, d_res, d_jac),
                    "gvx_small_factor_eval_dev")

    def marg_factor_eval(self, size, index, xoff, x0, params, J0, e0, jacobians=True):
        """MarginalizationFactor::Evaluate; J0 as an (r, r) array -> (residuals [r],
        jacobians [r * len(params)] (block b at r * xoff[b]) or None)."""
        sz, ix, xo = (np.ascontiguousarray(a, np.int32) for a in (size, index, xoff))
        J = np.ascontiguousarray(np.asarray(J0, np.float64).T)  # column-major data, as Eigen stores it
        r = J.shape[0]
        e = np.ascontiguousarray(e0, np.float64)
        z = np.ascontiguousarray(x0, np.float64)
        x = np.ascontiguousarray(params, np.float64)
        res = np.zeros(r)
        jac = np.zeros(r * x.size) if jacobians else None
        self._check(self._L.gvx_marg_factor_eval(self._h, r, sz.size, _ptr(sz), _ptr(ix), _ptr(xo), x.size, _ptr(z),
                                                 _ptr(x), _ptr(J), _ptr(e), _ptr(res), _ptr(jac)),
                    "gvx_marg_factor_eval")
        return res, jac

    # ---------------------------------------------------- marginalisation
    @staticmethod
    def _marg_struct(p):
        return (np.ascontiguousarray(p["nres"], np.int32), np.ascontiguousarray(p["blk_off"], np.int32),
                np.ascontiguousarray(p["blk"], np.int32), np.ascontiguousarray(p["res_off"], np.int64),
                np.ascontiguousarray(p["jac_off"], np.int64), np.ascontiguousarray(p["size"], np.int32),
                np.ascontiguousarray(p["index"], np.int32), int(p["m"]), int(p["L"]))

    def schur_solve(self, p, D=None):
        """One LM step of the window the way Ceres' DENSE_SCHUR takes it
        (gvx_schur_solve): p as marginalize's problem dict with the e-blocks
        (inverse depths) at local indices [0, m) -> dict(delta [L], S [r, r], info [2])."""
        nres, boff, blk, roff, joff, size, index, m, L = self._marg_struct(p)
        data = np.ascontiguousarray(p["data"], np.float64)
        Dv = None if D is None else np.ascontiguousarray(D, np.float64).reshape(L)
        r = L - m
        delta, S, info = np.zeros(L), np.zeros(max(r * r, 1)), np.zeros(2, np.int32)
        s = self._L.gvx_schur_solve(self._h, nres.size, _ptr(nres), _ptr(boff), _ptr(blk), _ptr(roff),
                                    _ptr(joff), _ptr(data), data.size, size.size, _ptr(size), _ptr(index), m,
                                    L, _ptr(Dv), _ptr(delta), _ptr(S), _ptr(info))
        if s != GVX_ERR_NUMERIC:  # a failed factorisation is a result (ok = False), not an error
            self._check(s, "gvx_schur_solve")
        return dict(delta=delta, S=S[:r * r].reshape(r, r).T.copy(), info=info, ok=s == GVX_OK)

    def schur_solve_dev(self, p, d_data, d_delta, d_D=None, d_S=None, d_info=None):
        """Device-pointer LM step (gvx_schur_solve_dev), async on the context stream."""
        nres, boff, blk, roff, joff, size, index, m, L = self._marg_struct(p)
        n_data = int(p["n_data"]) if "n_data" in p else int(np.asarray(p["data"]).size)
        self._check(self._L.gvx_schur_solve_dev(self._h, nres.size, _ptr(nres), _ptr(boff), _ptr(blk), _ptr(roff),
                                                _ptr(joff), d_data, n_data, size.size, _ptr(size), _ptr(index), m, L,
                                                d_D, d_delta, d_S, d_info), "gvx_schur_solve_dev")

    def marginalize(self, p):
        """MarginalizationInfo::marginalization() after preMarginalization on a
        problem dict (gvx.synth_ba.marg_problem) -> dict(J0 [r, r], e0, Hp [r, r],
        bp, eval, info [2])."""
        nres, boff, blk, roff, joff, size, index, m, L = self._marg_struct(p)
        data = np.ascontiguousarray(p["data"], np.float64)
        loss = p.get("loss")
        loss = None if loss is None else np.ascontiguousarray(loss, np.float64)
        r = L - m
        J0, Hp = np.zeros(max(r * r, 1)), np.zeros(max(r * r, 1))
        e0, bp, ev = np.zeros(max(r, 1)), np.zeros(max(r, 1)), np.zeros(max(r, 1))
        info = np.zeros(2, np.int32)
        self._check(self._L.gvx_marginalize(self._h, nres.size, _ptr(nres), _ptr(boff), _ptr(blk), _ptr(roff),
                                            _ptr(joff), _ptr(data), data.size, _ptr(loss), size.size, _ptr(size),
                                            _ptr(index), m, L, _ptr(J0), _ptr(e0), _ptr(Hp), _ptr(bp), _ptr(ev),
                                            _ptr(info)), "gvx_marginalize")
        cm = lambda a: a[:r * r].reshape(r, r).T.copy()  # column-major -> (r, r)
        return dict(J0=cm(J0), e0=e0[:r], Hp=cm(Hp), bp=bp[:r], eval=ev[:r], info=info)

    def marginalize_dev(self, p, d_data, d_J0, d_e0, d_Hp=None, d_bp=None, d_eval=None, d_info=None, d_loss=None):
        """Device-pointer marginalisation, async on the context stream (structure from p)."""
        nres, boff, blk, roff, joff, size, index, m, L = self._marg_struct(p)
        n_data = int(p["n_data"]) if "n_data" in p else int(np.asarray(p["data"]).size)
        self._check(self._L.gvx_marginalize_dev(self._h, nres.size, _ptr(nres), _ptr(boff), _ptr(blk), _ptr(roff),
                                                _ptr(joff), d_data, n_data, d_loss, size.size, _ptr(size),
                                                _ptr(index), m, L, d_J0, d_e0, d_Hp, d_bp, d_eval, d_info),
                    "gvx_marginalize_dev")

    def set_klt_phases(self, levels_per_phase: int, groups_per_chunk: int = 0):
        """gvx_set_klt_phases: the batched LK as phases of that many levels, one
        wave each, or 0 (default) = one wave per point group's whole chain;
        superchunks of groups_per_chunk groups (0 = unchanged, default 4096)."""
        self._check(self._L.gvx_set_klt_phases(self._h, levels_per_phase, groups_per_chunk), "gvx_set_klt_phases")

    def set_preint_path(self, path: int):
        """gvx_set_preint_path: PREINT_PATH_AUTO (the two-launch form: the per-step
        terms plus the chains by wave prefix products, then the covariance pass
        with sqrt_info in its epilogue) or PREINT_PATH_ONEPHASE (the single
        kernel; A/B and parity switch)."""
        self._check(self._L.gvx_set_preint_path(self._h, path), "gvx_set_preint_path")

    def set_marg_solver(self, solver: int):
        """gvx_set_marg_solver: MARG_SOLVER_EXACT (Eigen's eigen-solver, bit-exact
        vs the restatement) or MARG_SOLVER_FAST (Cholesky where no eigenvalue is
        dropped, the default)."""
        self._check(self._L.gvx_set_marg_solver(self._h, solver), "gvx_set_marg_solver")

    def sym_eigen(self, A):
        """Eigen::SelfAdjointEigenSolver on the device (lower triangle of A) ->
        (eigenvalues ascending, eigenvectors as columns, info)."""
        A = np.asarray(A, np.float64)
        n = A.shape[0]
        a = np.ascontiguousarray(A.T)
        w, V = np.zeros(max(n, 1)), np.zeros(max(n * n, 1))
        info = C.c_int32(0)
        self._check(self._L.gvx_sym_eigen(self._h, n, _ptr(a), n, _ptr(w), _ptr(V), C.byref(info)), "gvx_sym_eigen")
        return w[:n], V[:n * n].reshape(n, n).T.copy(), int(info.value)

    # ---------------------------------------------------- INS mechanization
    def ins_propagate(self, cfg: InsConfig, chains, states0):
        """insMechanization chained over each IMU series (misc.cc:174-229): chain i
        starts from states0[i] at chains[i][0] -> list of STATE_DTYPE arrays."""
        segs = [np.ascontiguousarray(s, dtype=IMU_DTYPE) for s in chains]
        n = len(segs)
        if n == 0:
            return []
        off = np.zeros(n + 1, np.int32)
        off[1:] = np.cumsum([len(s) for s in segs])
        imu = np.concatenate(segs)
        st0 = np.ascontiguousarray(states0, dtype=STATE_DTYPE).reshape(n)
        out = np.zeros(max(int(off[-1]), 1), STATE_DTYPE)
        self._check(self._L.gvx_ins_propagate(self._h, C.byref(cfg), n, _ptr(imu), _ptr(off), _ptr(st0),
                                              _ptr(out)), "gvx_ins_propagate")
        return [out[off[i]:off[i + 1]].copy() for i in range(n)]

    def ins_propagate_dev(self, cfg: InsConfig, n_chain, d_imu, d_off, d_state0, d_states):
        """Device-pointer INS chains (pointers as ints), async on the context stream."""
        self._check(self._L.gvx_ins_propagate_dev(self._h, C.byref(cfg), n_chain, d_imu, d_off, d_state0,
                                                  d_states), "gvx_ins_propagate_dev")

    def redo_ins_mechanization(self, cfg: InsConfig, updated, imu, states) -> int:
        """MISC::redoInsMechanization (misc.cc:231-284): states (STATE_DTYPE, len(imu))
        updated in place -> window index (0 = nothing done)."""
        imu = np.ascontiguousarray(imu, dtype=IMU_DTYPE)
        if states.dtype != STATE_DTYPE or not states.flags.c_contiguous or len(states) != len(imu):
            raise ValueError("states must be a contiguous STATE_DTYPE array of len(imu)")
        u = np.ascontiguousarray(updated, dtype=STATE_DTYPE).reshape(1)
        idx = C.c_int32()
        self._check(self._L.gvx_redo_ins_mechanization(self._h, C.byref(cfg), _ptr(u), len(imu), _ptr(imu),
                                                       _ptr(states), C.byref(idx)), "gvx_redo_ins_mechanization")
        return idx.value

    # ------------------------------------------------------------ hipGraphs
    def capture_begin(self):
        """Start capturing this context's stream (gvx_capture_begin)."""
        self._check(self._L.gvx_capture_begin(self._h), "gvx_capture_begin")

    def capture_end(self) -> "Graph":
        g = C.c_void_p()
        self._check(self._L.gvx_capture_end(self._h, C.byref(g)), "gvx_capture_end")
        return Graph(self, g)

    def capture_abort(self):
        """Discard an open capture (gvx_capture_abort)."""
        self._check(self._L.gvx_capture_abort(self._h), "gvx_capture_abort")

    def capture(self, fn, *args) -> "Graph":
        """Capture what fn(*args) enqueues into a graph; if fn raises, the capture
        is aborted (the context stays usable) and the error propagates."""
        self.capture_begin()
        try:
            fn(*args)
        except BaseException:
            self.capture_abort()
            raise
        return self.capture_end()

    def graph_launch(self, g: "Graph"):
        self._check(self._L.gvx_graph_launch(self._h, g.handle), "gvx_graph_launch")

    def copy_dev(self, d_dst: int, d_src: int, nbytes: int):
        """Device-to-device copy on the context stream (capturable)."""
        self._check(self._L.gvx_copy_dev(self._h, d_dst, d_src, nbytes), "gvx_copy_dev")

    def branch_begin(self):
        """Enqueue the following calls on a side branch (gvx_branch_begin)."""
        self._check(self._L.gvx_branch_begin(self._h), "gvx_branch_begin")

    def branch_end(self):
        """Back to the context stream, the branch running beside it (gvx_branch_end)."""
        self._check(self._L.gvx_branch_end(self._h), "gvx_branch_end")

    def branch_join(self):
        """The context stream waits for the branch (gvx_branch_join)."""
        self._check(self._L.gvx_branch_join(self._h), "gvx_branch_join")


class Graph:
    """A captured hipGraph of a context's stream; replay with launch()."""

    def __init__(self, ctx: Context, handle):
        self._ctx = ctx
        self._h = handle

    @property
    def handle(self):
        return self._h

    def launch(self):
        self._ctx.graph_launch(self)

    def destroy(self):
        if self._h:
            lib().gvx_graph_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def imu_series_from_to(imu, start, end):
    """MISC::getImuSeriesFromTo (misc.cc:330-384), host logic of the C ABI ->
    IMU_DTYPE array, or None when start or end is outside the window."""
    imu = np.ascontiguousarray(imu, dtype=IMU_DTYPE)
    out = np.zeros(len(imu) + 2, IMU_DTYPE)
    n = C.c_int32()
    s = lib().gvx_imu_series_from_to(_ptr(imu), len(imu), float(start), float(end), _ptr(out), C.byref(n))
    if s == -5:  # GVX_ERR_NOT_FOUND
        return None
    if s != GVX_OK:
        raise GvxError(f"gvx_imu_series_from_to: {lib().gvx_status_string(s).decode()}")
    return out[:n.value]


def earth_iewn(origin, local) -> np.ndarray:
    """Earth::iewn(station, p) as PreintegrationEarth::resetState computes it."""
    o = np.ascontiguousarray(origin, np.float64)
    l_ = np.ascontiguousarray(local, np.float64)
    out = np.zeros(3)
    lib().gvx_earth_iewn(_ptr(o), _ptr(l_), _ptr(out))
    return out


class FactorSet:
    """Two-phase factor evaluation (gvx_factor_set_* / gvx_factors_prepare /
    gvx_factor_read_*): the Ceres EvaluationCallback pattern.  `blocks` are the
    caller's float64 parameter blocks; prepare() re-reads them in place, like
    PrepareForEvaluation after Ceres has written a candidate point."""

    RP_SIZES = (7, 7, 7, 1, 1)
    PF_SIZES = (7, 9, 7, 9)

    def __init__(self, ctx: "Context", blocks, reproj_consts=None, r_blocks=None, pre=None, pn=None,
                 pn_off=None, p_blocks=None):
        self._ctx = ctx
        self._blocks = [b for b in blocks]
        for b in self._blocks:
            if not (isinstance(b, np.ndarray) and b.dtype == np.float64 and b.flags.c_contiguous):
                raise GvxError("parameter blocks must be C-contiguous float64 arrays")
        nb = len(self._blocks)
        self._ptrs = (C.c_void_p * nb)(*[b.ctypes.data for b in self._blocks])
        self._sizes = np.array([b.size for b in self._blocks], np.int32)
        rc = np.ascontiguousarray(reproj_consts if reproj_consts is not None else np.zeros(0, REPROJ_DTYPE),
                                  dtype=REPROJ_DTYPE)
        self.n_reproj = rc.shape[0]
        rb = np.ascontiguousarray(r_blocks if r_blocks is not None else np.zeros((0, 5)), np.int32).reshape(-1, 5)
        pr = np.ascontiguousarray(pre if pre is not None else np.zeros(0, PREINT_DTYPE), dtype=PREINT_DTYPE)
        self.n_preint = pr.shape[0]
        pb = np.ascontiguousarray(p_blocks if p_blocks is not None else np.zeros((0, 4)), np.int32).reshape(-1, 4)
        pnn = np.ascontiguousarray(pn if pn is not None else np.zeros((0, 4)), np.float64).reshape(-1, 4)
        pno = np.ascontiguousarray(pn_off if pn_off is not None else np.zeros(self.n_preint), np.int32)
        h = C.c_void_p()
        ctx._check(ctx._L.gvx_factor_set_create(ctx._h, nb, self._ptrs, _ptr(self._sizes), self.n_reproj, _ptr(rc),
                                                _ptr(rb), self.n_preint, _ptr(pr), _ptr(pnn), pnn.shape[0],
                                                _ptr(pno), _ptr(pb), C.byref(h)), "gvx_factor_set_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._ctx._L.gvx_factor_set_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def prepare(self, jacobians: bool = True):
        self._ctx._check(self._ctx._L.gvx_factors_prepare(self._h, 1 if jacobians else 0), "gvx_factors_prepare")

    def _read(self, fn, i, n_res, sizes, jacobians):
        res = np.zeros(n_res)
        if jacobians is False or jacobians is None:
            s = fn(self._h, i, _ptr(res), None)
            if s != GVX_OK:
                raise GvxError(f"factor read {i}: {self._ctx._L.gvx_status_string(s).decode()}")
            return res, None
        want = [True] * len(sizes) if jacobians is True else list(jacobians)
        J = [np.zeros((n_res, k)) if w else None for w, k in zip(want, sizes)]
        arr = (C.c_void_p * len(sizes))(*[j.ctypes.data if j is not None else None for j in J])
        s = fn(self._h, i, _ptr(res), arr)
        if s != GVX_OK:
            raise GvxError(f"factor read {i}: {self._ctx._L.gvx_status_string(s).decode()}")
        return res, J

    def read_reproj(self, i: int, jacobians=True):
        """(residuals[2], [J_pose_ref 2x7, J_pose_obs 2x7, J_ext 2x7, J_invdepth 2x1, J_td 2x1]);
        jacobians: True, False, or a per-block list of booleans (False -> null block)."""
        return self._read(self._ctx._L.gvx_factor_read_reproj, i, 2, self.RP_SIZES, jacobians)

    def read_preint(self, i: int, jacobians=True):
        """(residuals[15], [J_pose0 15x7, J_mix0 15x9, J_pose1 15x7, J_mix1 15x9])."""
        return self._read(self._ctx._L.gvx_factor_read_preint, i, 15, self.PF_SIZES, jacobians)
