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


class InsConfig(C.Structure):
    """IntegrationConfiguration as insMechanization reads it (integration_state.h:91-99)."""
    _fields_ = [("iswithearth", C.c_int), ("gravity", C.c_double * 3), ("iewn", C.c_double * 3)]

    @classmethod
    def make(cls, iswithearth, gravity, iewn=(0.0, 0.0, 0.0)):
        c = cls()
        c.iswithearth = int(bool(iswithearth))
        for i in range(3):
            c.gravity[i] = float(gravity[i])
            c.iewn[i] = float(iewn[i])
        return c


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


class Camera(C.Structure):
    """Camera intrinsics + distortion (tracking/camera.cc:25-46)."""
    _fields_ = [(k, C.c_double) for k in ("fx", "fy", "cx", "cy", "skew", "k1", "k2", "p1", "p2", "k3")] + \
               [("width", C.c_int), ("height", C.c_int)]


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
        L.orc_set_lk_accum.argtypes = [C.c_int]
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
        L.orc_reproj_eval_batch.argtypes = [C.c_int, P, P, P, P, P, C.c_int]
        L.orc_preint_factor_eval_batch.argtypes = [C.c_int, P, P, P, P, P, C.c_int]
        L.orc_pose_plus.argtypes = [P, P, P]
        L.orc_clahe_luts.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int, C.c_int, P]
        L.orc_clahe.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int, C.c_int, P, C.c_int]
        L.orc_bgr2gray.argtypes = [P, C.c_int, C.c_int, C.c_int, P, C.c_int]
        L.orc_hist_mean.argtypes = [P, C.c_int, C.c_int, C.c_int]
        L.orc_hist_mean.restype = C.c_double
        IC = C.POINTER(InsConfig)
        L.orc_ins_mechanization.argtypes = [IC, P, P, C.POINTER(State)]
        L.orc_ins_propagate.argtypes = [IC, P, C.c_int, C.POINTER(State), P]
        L.orc_redo_ins_mechanization.argtypes = [IC, C.POINTER(State), P, C.c_int, P]
        L.orc_redo_ins_mechanization.restype = C.c_int
        L.orc_imu_series_from_to.argtypes = [P, C.c_int, C.c_double, C.c_double, P]
        L.orc_imu_series_from_to.restype = C.c_int
        L.orc_ins_window_index.argtypes = [P, C.c_int, C.c_double]
        L.orc_ins_window_index.restype = C.c_int
        L.orc_need_interpolation.argtypes = [P, P, C.c_double]
        L.orc_need_interpolation.restype = C.c_int
        L.orc_small_factor_eval.argtypes = [C.c_int, C.c_int, P, P, P, P, P]
        L.orc_small_factor_eval.restype = C.c_int
        L.orc_marg_factor_eval.argtypes = [C.c_int, C.c_int, P, P, P, P, P, P, P, P, P]
        L.orc_sym_eigen.argtypes = [C.c_int, P, C.c_int, P, P]
        L.orc_sym_eigen.restype = C.c_int
        L.orc_marg_construct.argtypes = [C.c_int, P, P, P, P, P, P, P, P, C.c_int, P, P]
        L.orc_marg_schur.argtypes = [C.c_int, C.c_int, P, P, P, P]
        L.orc_marg_schur.restype = C.c_int
        L.orc_marg_linearize.argtypes = [C.c_int, P, P, P, P, P]
        L.orc_marg_linearize.restype = C.c_int
        L.orc_find_fundamental_ransac.argtypes = [C.c_int, P, P, C.c_double, C.c_double, C.c_int, P, P,
                                                  C.POINTER(C.c_int)]
        L.orc_find_fundamental_ransac.restype = C.c_int
        L.orc_run7point.argtypes = [P, P, P]
        L.orc_run7point.restype = C.c_int
        L.orc_solve_cubic.argtypes = [P, P]
        L.orc_solve_cubic.restype = C.c_int
        L.orc_fm_error.argtypes = [C.c_int, P, P, P, P]
        L.orc_ransac_update_num_iters.argtypes = [C.c_double, C.c_double, C.c_int, C.c_int]
        L.orc_ransac_update_num_iters.restype = C.c_int
        L.orc_cvrng_next.argtypes = [C.POINTER(C.c_uint64)]
        L.orc_cvrng_next.restype = C.c_uint
        CP = C.POINTER(Camera)
        L.orc_undistort_points.argtypes = [CP, C.c_int, P, P]
        L.orc_distort_points.argtypes = [CP, C.c_int, P, P]
        L.orc_predict_rotated.argtypes = [CP, P, C.c_int, P, P]
        L.orc_project_points.argtypes = [CP, P, P, C.c_int, P, P]
        L.orc_point_velocity.argtypes = [CP, C.c_int, P, P, C.c_double, P]
        L.orc_keypoint_parallax.argtypes = [CP, P, P, C.c_int, P, P, P]
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


ACC_EXACT, ACC_F32, ACC_F32X4 = 0, 1, 2


class lk_accum:
    """Context manager selecting LK's window-sum accumulation order (klt.c
    ORC_ACC_*): the exact int64 default, or OpenCV 4.x's fp32 scalar / 4-lane
    SIMD orders for the parity-sensitivity experiment."""

    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        lib().orc_set_lk_accum(self.mode)
        return self

    def __exit__(self, *exc):
        lib().orc_set_lk_accum(ACC_EXACT)
        return False


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


# ------------------------------------------------------------- preintegration
IMU_DTYPE = np.dtype([("time", "f8"), ("dt", "f8"), ("dtheta", "f8", 3), ("dvel", "f8", 3), ("odovel", "f8")])


def imu_params(acc_vrw, gyr_arw, gyr_bias_std, acc_bias_std, corr_time, gravity):
    return ImuParams(acc_vrw, gyr_arw, gyr_bias_std, acc_bias_std, corr_time, gravity)


def make_state(time=0.0, p=(0, 0, 0), q=(0, 0, 0, 1), v=(0, 0, 0), bg=(0, 0, 0), ba=(0, 0, 0)):
    s = State()
    s.time = time
    for name, val in (("p", p), ("q", q), ("v", v), ("bg", bg), ("ba", ba)):
        arr = getattr(s, name)
        for i, x in enumerate(val):
            arr[i] = float(x)
    return s


def state_dict(s: State):
    return dict(time=s.time, p=np.array(s.p[:]), q=np.array(s.q[:]), v=np.array(s.v[:]),
                bg=np.array(s.bg[:]), ba=np.array(s.ba[:]))


class PreintSeg:
    """Owns an orc_preint (freed on deletion)."""

    def __init__(self, variant, prm, imu: np.ndarray, state0: State, iewn=(0.0, 0.0, 0.0)):
        self.imu = np.ascontiguousarray(imu, dtype=IMU_DTYPE)
        self.prm = prm
        self.iewn = np.asarray(iewn, np.float64)
        self.s = Preint()
        lib().orc_preint_integrate(C.byref(self.s), variant, C.byref(prm), _p(self.imu), len(self.imu),
                                   C.byref(state0), _p(self.iewn))

    def reintegrate(self, state: State, iewn=None):
        if iewn is not None:
            self.iewn = np.asarray(iewn, np.float64)
        lib().orc_preint_reintegrate(C.byref(self.s), C.byref(self.prm), _p(self.imu), C.byref(state),
                                     _p(self.iewn))

    def __del__(self):
        try:
            lib().orc_preint_free(C.byref(self.s))
        except Exception:
            pass

    @property
    def jacobian(self):
        return np.array(self.s.jacobian[:]).reshape(15, 15)

    @property
    def covariance(self):
        return np.array(self.s.covariance[:]).reshape(15, 15)

    @property
    def pn(self):
        m = self.s.m - 1
        return np.ctypeslib.as_array(self.s.pn, shape=(max(m, 1) * 4,))[:m * 4].reshape(m, 4).copy()

    def delta(self):
        return state_dict(self.s.delta)

    def current(self):
        return state_dict(self.s.current)

    def evaluate(self, pose0, mix0, pose1, mix1, jacobians=True):
        blocks = [np.ascontiguousarray(b, np.float64) for b in (pose0, mix0, pose1, mix1)]
        params = (C.c_void_p * 4)(*[b.ctypes.data for b in blocks])
        res = np.zeros(15)
        if not jacobians:
            lib().orc_preint_factor_eval(C.byref(self.s), params, _p(res), None)
            return res, None
        J = [np.zeros((15, 7)), np.zeros((15, 9)), np.zeros((15, 7)), np.zeros((15, 9))]
        jp = (C.c_void_p * 4)(*[j.ctypes.data for j in J])
        lib().orc_preint_factor_eval(C.byref(self.s), params, _p(res), jp)
        return res, J


def earth_iewn(origin, local):
    o = np.ascontiguousarray(origin, np.float64)
    l_ = np.ascontiguousarray(local, np.float64)
    out = np.zeros(3)
    lib().orc_earth_iewn(_p(o), _p(l_), _p(out))
    return out


# ------------------------------------------------------------- reprojection
def reproj_const(pts0, pts1, vel0, vel1, td0, td1, std):
    c = ReprojConst()
    for name, val in (("pts0", pts0), ("pts1", pts1), ("vel0", vel0), ("vel1", vel1)):
        arr = getattr(c, name)
        for i in range(3):
            arr[i] = float(val[i])
    c.td0, c.td1, c.std = float(td0), float(td1), float(std)
    return c


def reproj_eval(c: ReprojConst, pose_i, pose_j, ext, invdepth, td, jacobians=True):
    blocks = [np.ascontiguousarray(b, np.float64).reshape(-1) for b in (pose_i, pose_j, ext, [invdepth], [td])]
    params = (C.c_void_p * 5)(*[b.ctypes.data for b in blocks])
    res = np.zeros(2)
    if not jacobians:
        lib().orc_reproj_eval(C.byref(c), params, _p(res), None)
        return res, None
    J = [np.zeros((2, 7)), np.zeros((2, 7)), np.zeros((2, 7)), np.zeros((2, 1)), np.zeros((2, 1))]
    jp = (C.c_void_p * 5)(*[j.ctypes.data for j in J])
    lib().orc_reproj_eval(C.byref(c), params, _p(res), jp)
    return res, J


def pose_plus(x, delta):
    x = np.ascontiguousarray(x, np.float64)
    d = np.ascontiguousarray(delta, np.float64)
    out = np.zeros(7)
    lib().orc_pose_plus(_p(x), _p(d), _p(out))
    return out


# ------------------------------------------------------------- detection
def block_grid(w, h, params=None):
    g = BlockGrid()
    lib().orc_block_grid_make(w, h, C.byref(params or DetectParams.default()), C.byref(g))
    return g


def mask_circles(w, h, xy, radius):
    mask = np.full((h, w), 255, np.uint8)
    xy = np.ascontiguousarray(xy, np.float32).reshape(-1, 2)
    lib().orc_mask_circles(_p(mask), w, h, _p(xy), xy.shape[0], radius)
    return mask


def corner_min_eigen_val(img, x0, y0, rw, rh):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    eig = np.zeros((rh, rw), np.float32)
    lib().orc_corner_min_eigen_val(_p(img), w, h, w, x0, y0, rw, rh, _p(eig))
    return eig


def good_features_to_track(img, x0, y0, rw, rh, mask_roi, max_corners, quality, min_distance):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    m = None if mask_roi is None else np.ascontiguousarray(mask_roi, np.uint8)
    out = np.zeros((max(max_corners, 1) if max_corners > 0 else rw * rh, 2), np.float32)
    n = lib().orc_good_features_to_track(_p(img), w, h, w, x0, y0, rw, rh, _p(m),
                                         0 if m is None else m.shape[1], max_corners, quality,
                                         min_distance, _p(out))
    return out[:n].copy()


def features_detection(img, count_xy=None, mask_xy=None, ismask=True, n_existing=0, params=None):
    """-> (corners [n,2] or None on early exit, per-block counts)."""
    p = params or DetectParams.default()
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    g = block_grid(w, h, p)
    cxy = np.zeros((0, 2), np.float32) if count_xy is None else np.ascontiguousarray(count_xy, np.float32).reshape(-1, 2)
    mxy = np.zeros((0, 2), np.float32) if mask_xy is None else np.ascontiguousarray(mask_xy, np.float32).reshape(-1, 2)
    out = np.zeros((max(g.block_cnts * max(g.max_block_features, 1), 1), 2), np.float32)
    blk = np.zeros(max(g.block_cnts, 1), np.int32)
    n = lib().orc_features_detection(_p(img), w, h, w, _p(cxy), cxy.shape[0], _p(mxy), mxy.shape[0],
                                     1 if ismask else 0, n_existing, C.byref(p), _p(out), _p(blk))
    if n < 0:
        return None, blk[:0]
    return out[:n].copy(), blk[:g.block_cnts]


def reproj_eval_batch(consts: np.ndarray, params, offs, jacobians=True, nthreads=1):
    """n reprojection factors (consts: structured array with the ReprojConst
    fields) -> (residuals [n,2], jacobians [n,46] or None)."""
    cs = np.ascontiguousarray(consts)
    n = cs.shape[0]
    prm = np.ascontiguousarray(params, np.float64)
    o = np.ascontiguousarray(offs, np.int32).reshape(n, 5)
    res = np.zeros((n, 2))
    jac = np.zeros((n, 46)) if jacobians else None
    lib().orc_reproj_eval_batch(n, _p(cs), _p(prm), _p(o), _p(res), _p(jac), nthreads)
    return res, jac


def preint_factor_eval_batch(segs, params, offs, jacobians=True, nthreads=1):
    """n preintegration factors over PreintSeg objects -> (residuals [n,15], jacobians [n,480] or None)."""
    n = len(segs)
    ptrs = (C.c_void_p * n)(*[C.addressof(s.s) for s in segs])
    prm = np.ascontiguousarray(params, np.float64)
    o = np.ascontiguousarray(offs, np.int32).reshape(n, 4)
    res = np.zeros((n, 15))
    jac = np.zeros((n, 480)) if jacobians else None
    lib().orc_preint_factor_eval_batch(n, C.cast(ptrs, C.c_void_p), _p(prm), _p(o), _p(res), _p(jac), nthreads)
    return res, jac


# ------------------------------------------------------------------ preprocessing
def bgr2gray(bgr: np.ndarray) -> np.ndarray:
    """cv::cvtColor(COLOR_BGR2GRAY) of an h x w x 3 u8 image (clahe.c)."""
    bgr = np.ascontiguousarray(bgr, np.uint8)
    h, w = bgr.shape[:2]
    out = np.zeros((h, w), np.uint8)
    lib().orc_bgr2gray(_p(bgr), w, h, 3 * w, _p(out), w)
    return out


def clahe(img: np.ndarray, clip_limit=3.0, tiles=(21, 21)) -> np.ndarray:
    """cv::createCLAHE(clip_limit, Size(tiles))->apply(img) (tracking.cc:63, :139)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.empty_like(img)
    lib().orc_clahe(_p(img), w, h, w, clip_limit, tiles[0], tiles[1], _p(out), w)
    return out


def clahe_luts(img: np.ndarray, clip_limit=3.0, tiles=(21, 21)) -> np.ndarray:
    """The per-tile LUTs (tiles_y*tiles_x x 256) of CLAHE_CalcLut_Body."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.empty((tiles[1] * tiles[0], 256), np.uint8)
    lib().orc_clahe_luts(_p(img), w, h, w, clip_limit, tiles[0], tiles[1], _p(out))
    return out


def hist_mean(img: np.ndarray) -> float:
    """Tracking::calculateHistigram (tracking.cc:88-105)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    return float(lib().orc_hist_mean(_p(img), w, h, w))


# ------------------------------------------------------------------ camera ops
def _xy(a):
    return np.ascontiguousarray(a, np.float32).reshape(-1, 2)


def undistort_points(cam: Camera, pts):
    p = _xy(pts)
    out = np.empty_like(p)
    lib().orc_undistort_points(C.byref(cam), len(p), _p(p), _p(out))
    return out


def distort_points(cam: Camera, pts):
    p = _xy(pts)
    out = np.empty_like(p)
    lib().orc_distort_points(C.byref(cam), len(p), _p(p), _p(out))
    return out


def predict_rotated(cam: Camera, r_cur_pre, pts):
    p = _xy(pts)
    R = np.ascontiguousarray(r_cur_pre, np.float64).reshape(9)
    out = np.empty_like(p)
    lib().orc_predict_rotated(C.byref(cam), _p(R), len(p), _p(p), _p(out))
    return out


def project_points(cam: Camera, R, t, pw):
    R = np.ascontiguousarray(R, np.float64).reshape(9)
    t = np.ascontiguousarray(t, np.float64).reshape(3)
    pw = np.ascontiguousarray(pw, np.float64).reshape(-1, 3)
    out = np.empty((len(pw), 2), np.float32)
    lib().orc_project_points(C.byref(cam), _p(R), _p(t), len(pw), _p(pw), _p(out))
    return out


def point_velocity(cam: Camera, pre, cur, dt):
    a, b = _xy(pre), _xy(cur)
    out = np.empty((len(a), 2), np.float64)
    lib().orc_point_velocity(C.byref(cam), len(a), _p(a), _p(b), dt, _p(out))
    return out


def keypoint_parallax(cam: Camera, R0, R1, ref, cur):
    a, b = _xy(ref), _xy(cur)
    R0 = np.ascontiguousarray(R0, np.float64).reshape(9)
    R1 = np.ascontiguousarray(R1, np.float64).reshape(9)
    out = np.empty(len(a), np.float64)
    lib().orc_keypoint_parallax(C.byref(cam), _p(R0), _p(R1), len(a), _p(a), _p(b), _p(out))
    return out


# ------------------------------------------------------------------ INS mechanization
STATE_DTYPE = np.dtype([("time", "f8"), ("p", "f8", 3), ("q", "f8", 4), ("v", "f8", 3), ("bg", "f8", 3),
                        ("ba", "f8", 3)])


def _state_array(n):
    return np.zeros(n, STATE_DTYPE)


def ins_propagate(cfg: InsConfig, imu, state0: State):
    """insMechanization chained over imu[0..m) from state0 (at imu[0].time) -> m states."""
    imu = np.ascontiguousarray(imu, dtype=IMU_DTYPE)
    out = _state_array(len(imu))
    lib().orc_ins_propagate(C.byref(cfg), _p(imu), len(imu), C.byref(state0), _p(out))
    return out


def redo_ins_mechanization(cfg: InsConfig, updated: State, imu, states):
    """MISC::redoInsMechanization on a window (imu[n], states[n], updated in place) -> index."""
    imu = np.ascontiguousarray(imu, dtype=IMU_DTYPE)
    assert states.dtype == STATE_DTYPE and states.flags.c_contiguous
    return int(lib().orc_redo_ins_mechanization(C.byref(cfg), C.byref(updated), _p(imu), len(imu), _p(states)))


def imu_series_from_to(imu, start, end):
    imu = np.ascontiguousarray(imu, dtype=IMU_DTYPE)
    out = np.zeros(len(imu) + 2, IMU_DTYPE)
    m = lib().orc_imu_series_from_to(_p(imu), len(imu), start, end, _p(out))
    return None if m < 0 else out[:m]


def ins_window_index(imu, n, t):
    """MISC::getInsWindowIndex (misc.cc:40-83): first index with time > t, 0 = none."""
    imu = np.ascontiguousarray(imu, dtype=IMU_DTYPE)
    return int(lib().orc_ins_window_index(_p(imu), n, t))


# ------------------------------------------------ remaining window factors
SMALL_FACTOR_DIMS = {0: (3, 7, 9), 1: (6, 9, 0), 2: (6, 7, 13), 3: (9, 9, 18)}  # GNSS, IMU_ERROR, POSE/MIX_PRIOR


def small_factor_eval(kind, consts, params, offs, jacobians=True):
    """GnssFactor / ImuErrorFactor / ImuPosePriorFactor / ImuMixPriorFactor batch
    (aux_factors.c) -> (residuals [n, R], jacobians [n, R*P] or None)."""
    R, P, NC = SMALL_FACTOR_DIMS[kind]
    o = np.ascontiguousarray(offs, np.int32).reshape(-1)
    n = o.size
    cs = np.ascontiguousarray(consts, np.float64).reshape(-1) if NC else np.zeros(1)
    prm = np.ascontiguousarray(params, np.float64).reshape(-1)
    res = np.zeros((n, R))
    jac = np.zeros((n, R * P)) if jacobians else None
    assert lib().orc_small_factor_eval(kind, n, _p(cs), _p(prm), _p(o), _p(res), _p(jac)) == 0
    return res, jac


def marg_factor_eval(size, index, xoff, x0, params, J0, e0, jacobians=True):
    """MarginalizationFactor::Evaluate (aux_factors.c); J0 given as an (r, r)
    array -> (residuals [r], jacobians [r * sum(size)] or None)."""
    sz = np.ascontiguousarray(size, np.int32)
    ix = np.ascontiguousarray(index, np.int32)
    xo = np.ascontiguousarray(xoff, np.int32)
    J = np.ascontiguousarray(np.asarray(J0, np.float64).T)  # column-major data, as Eigen stores it
    r = J.shape[0]
    e = np.ascontiguousarray(e0, np.float64)
    z = np.ascontiguousarray(x0, np.float64)
    x = np.ascontiguousarray(params, np.float64)
    res = np.zeros(r)
    jac = np.zeros(r * int(sz.sum())) if jacobians else None
    lib().orc_marg_factor_eval(r, sz.size, _p(sz), _p(ix), _p(xo), _p(z), _p(x), _p(J), _p(e), _p(res), _p(jac))
    return res, jac


# ------------------------------------------------------ marginalisation
def sym_eigen(A):
    """Eigen::SelfAdjointEigenSolver (marg.c): lower triangle of A read ->
    (eigenvalues ascending, eigenvectors as columns, info)."""
    A = np.asarray(A, np.float64)
    n = A.shape[0]
    a = np.ascontiguousarray(A.T)  # column-major data
    w = np.zeros(max(n, 1))
    V = np.zeros(max(n * n, 1))
    info = lib().orc_sym_eigen(n, _p(a), n, _p(w), _p(V))
    return w[:n], V[:n * n].reshape(n, n).T.copy(), int(info)


def marg_construct(problem):
    """constructEquation (marg.c) over a problem dict (gvx.synth_ba.marg_problem:
    nres, blk_off, blk, res_off, jac_off, data, loss, size, index, m, L) -> (H0 [L, L], b0 [L])."""
    p = problem
    L = int(p["L"])
    H0 = np.zeros(L * L)
    b0 = np.zeros(L)
    nres = np.ascontiguousarray(p["nres"], np.int32)
    boff = np.ascontiguousarray(p["blk_off"], np.int32)
    blk = np.ascontiguousarray(p["blk"], np.int32)
    foff = np.ascontiguousarray(p["res_off"], np.int64)
    assert np.array_equal(np.asarray(p["jac_off"]), foff + nres), "oracle layout: Jacobians follow the residuals"
    data = np.ascontiguousarray(p["data"], np.float64)
    loss = p.get("loss")
    loss = None if loss is None else np.ascontiguousarray(loss, np.float64)
    size = np.ascontiguousarray(p["size"], np.int32)
    index = np.ascontiguousarray(p["index"], np.int32)
    lib().orc_marg_construct(nres.size, _p(nres), _p(boff), _p(blk), _p(foff), _p(data), _p(loss), _p(size),
                             _p(index), L, _p(H0), _p(b0))
    return H0.reshape(L, L).T.copy(), b0


def marg_schur(H0, b0, m):
    """schurElimination (marg.c) -> (Hp [r, r], bp [r], info)."""
    H0 = np.asarray(H0, np.float64)
    L = H0.shape[0]
    r = L - m
    h = np.ascontiguousarray(H0.T)
    b = np.ascontiguousarray(b0, np.float64)
    Hp = np.zeros(max(r * r, 1))
    bp = np.zeros(max(r, 1))
    info = lib().orc_marg_schur(L, m, _p(h), _p(b), _p(Hp), _p(bp))
    return Hp[:r * r].reshape(r, r).T.copy(), bp[:r], int(info)


def marg_linearize(Hp, bp):
    """linearization (marg.c) -> (J0 [r, r], e0 [r], eigenvalues [r], info)."""
    Hp = np.asarray(Hp, np.float64)
    r = Hp.shape[0]
    h = np.ascontiguousarray(Hp.T)
    b = np.ascontiguousarray(bp, np.float64)
    J0 = np.zeros(max(r * r, 1))
    e0 = np.zeros(max(r, 1))
    ev = np.zeros(max(r, 1))
    info = lib().orc_marg_linearize(r, _p(h), _p(b), _p(J0), _p(e0), _p(ev))
    return J0[:r * r].reshape(r, r).T.copy(), e0[:r], ev[:r], int(info)


class FactorEvaluator:
    """synth_ba.make_marg_problem's evaluator on the CPU restatement (tests only)."""

    def reproj(self, consts, params, offs):
        return reproj_eval_batch(consts, params, offs)

    def preint(self, imu, st, p0, m0, p1, m1):
        from gvx import synth_ba  # the synthetic IMU's noise parameters
        s = make_state(float(st["time"]), st["p"], st["q"], st["v"], st["bg"], st["ba"])
        seg = PreintSeg(2, imu_params(*synth_ba.imu_params()), imu, s, np.zeros(3))
        r, J = seg.evaluate(p0, m0, p1, m1)
        return r, np.concatenate([j.ravel() for j in J])

    def gnss(self, consts, pose):
        res, jac = small_factor_eval(0, np.asarray(consts).reshape(1, -1), pose, np.array([0], np.int32))
        return res[0], jac[0]

    def marg(self, size, index, xoff, x0, x, J0, e0):
        return marg_factor_eval(size, index, xoff, x0, x, J0, e0)


# ------------------------------------------------ findFundamentalMat(FM_RANSAC)
def find_fundamental_ransac(p1, p2, thresh=1.5, confidence=0.99, max_iters=1000):
    """cv::findFundamentalMat(p1, p2, FM_RANSAC, thresh, confidence) (fmat.c) ->
    (result, mask u8 [n], F [3, 3] or None, iterations)."""
    a = np.ascontiguousarray(p1, np.float32).reshape(-1, 2)
    b = np.ascontiguousarray(p2, np.float32).reshape(-1, 2)
    n = a.shape[0]
    mask = np.zeros(max(n, 1), np.uint8)
    F = np.zeros(9)
    it = C.c_int(0)
    r = lib().orc_find_fundamental_ransac(n, _p(a), _p(b), thresh, confidence, max_iters, _p(mask), _p(F),
                                          C.byref(it))
    return int(r), mask[:n], (F.reshape(3, 3) if r > 0 else None), int(it.value)


def run7point(p1, p2):
    a = np.ascontiguousarray(p1, np.float32).reshape(7, 2)
    b = np.ascontiguousarray(p2, np.float32).reshape(7, 2)
    F = np.zeros(27)
    n = lib().orc_run7point(_p(a), _p(b), _p(F))
    return [F[9 * k:9 * k + 9].reshape(3, 3) for k in range(max(n, 0))]


def solve_cubic(coeffs):
    c = np.ascontiguousarray(coeffs, np.float64)
    r = np.zeros(3)
    n = lib().orc_solve_cubic(_p(c), _p(r))
    return n, r


def fm_error(p1, p2, F):
    a = np.ascontiguousarray(p1, np.float32).reshape(-1, 2)
    b = np.ascontiguousarray(p2, np.float32).reshape(-1, 2)
    f = np.ascontiguousarray(F, np.float64).reshape(9)
    err = np.zeros(a.shape[0], np.float32)
    lib().orc_fm_error(a.shape[0], _p(a), _p(b), _p(f), _p(err))
    return err


def ransac_update_num_iters(p, ep, model_points, max_iters):
    return int(lib().orc_ransac_update_num_iters(p, ep, model_points, max_iters))


def cvrng_sequence(state, n):
    s = C.c_uint64(state)
    return [int(lib().orc_cvrng_next(C.byref(s))) for _ in range(n)]
