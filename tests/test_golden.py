"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py from
the CPU restatement).  CPU: the oracle still reproduces every fixture exactly
(regression pin of the restatement; the reference itself holds no fixtures for
this path -- parity unpinned against OpenCV/Eigen).
GPU: libgvx reproduces the same vectors -- bit-exact for pyramids, LK, FB,
compaction, detection and the reprojection factor; fp64 preintegration within
1e-10 and the preintegration factor within 1e-9 (ocml vs glibc sin/cos)."""
import glob
import os

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NORMAL, EARTH = 0, 2


def load(name):
    return np.load(os.path.join(HERE, name), allow_pickle=False)


def cases(prefix):
    return sorted(os.path.basename(f) for f in glob.glob(os.path.join(HERE, prefix + "*.npz")))


def _close(g, o, what, rtol):
    g, o = np.asarray(g, np.float64), np.asarray(o, np.float64)
    scale = max(np.abs(o).max(), 1e-300)
    assert np.abs(g - o).max() <= rtol * scale, f"{what}: {np.abs(g - o).max():.3e} vs {scale:.3e}"


def _imu(z):
    from gvx import synth_ba
    return np.ascontiguousarray(z["imu"]).view(synth_ba.IMU_DTYPE).reshape(-1)


def _state_fields(z):
    s = z["state0"]
    return dict(time=s[0], p=s[1:4], q=s[4:8], v=s[8:11], bg=s[11:14], ba=s[14:17])


def test_fixtures_present():
    assert len(cases("klt_")) >= 3 and cases("detect_") and len(cases("preint_")) >= 3 and cases("reproj_")


# ------------------------------------------------------------------ CPU: oracle
@pytest.mark.parametrize("name", cases("klt_"))
def test_oracle_klt_golden(orc, name):
    z = load(name)
    L = int(z["levels"])
    for k, lv in enumerate(orc.build_pyramid(z["I"], L)):
        assert np.array_equal(lv, z[f"level{k}"]), f"level {k}"
    p = orc.KltParams.default(max_level=L)
    nxt, st, err = orc.calc_optical_flow_pyr_lk(z["I"], z["J"], z["prev"], z["init"], p)
    assert np.array_equal(nxt, z["next"]) and np.array_equal(st, z["status"]) and np.array_equal(err, z["err"])
    h, w = z["I"].shape
    fb = orc.klt_fb(z["I"], z["J"], z["prev"], z["init"], w, h, params=p, reuse_pyramids=True)
    for k in ("next", "back", "st_f", "st_b", "keep"):
        assert np.array_equal(fb[k], z["fb_" + k]), k
    assert np.array_equal(fb["kept_idx"], z["fb_kept"])


def test_oracle_detect_golden(orc):
    z = load("detect_320x140.npz")
    prm = orc.DetectParams.default(max_features=int(z["max_features"]))
    c, b = orc.features_detection(z["img"], z["tracked"], z["tracked"], True, len(z["tracked"]), prm)
    assert np.array_equal(c, z["corners"]) and np.array_equal(np.asarray(b, np.int32), z["blocks"])


@pytest.mark.parametrize("name", cases("preint_"))
def test_oracle_preint_golden(orc, name):
    z = load(name)
    s = _state_fields(z)
    seg = orc.PreintSeg(int(z["variant"]), orc.imu_params(*z["prm"]), _imu(z),
                        orc.make_state(float(s["time"]), s["p"], s["q"], s["v"], s["bg"], s["ba"]), z["iewn"])
    d, c = seg.delta(), seg.current()
    for k in ("p", "q", "v"):
        assert np.array_equal(d[k], z["delta_" + k]) and np.array_equal(c[k], z["current_" + k]), k
    assert np.array_equal(seg.jacobian, z["jacobian"]) and np.array_equal(seg.covariance, z["covariance"])
    prm = z["params"]
    r, J = seg.evaluate(prm[:7], prm[7:16], prm[16:23], prm[23:32])
    assert np.array_equal(r, z["residual"])
    assert np.array_equal(np.concatenate([x.ravel() for x in J]), z["jac"])


def test_oracle_reproj_golden(orc):
    z = load("reproj_3kf_16lm.npz")
    prm = z["params"]
    for i, (c, o) in enumerate(zip(z["consts"], z["offs"])):
        rc = orc.reproj_const(c[0:3], c[3:6], c[6:9], c[9:12], c[12], c[13], c[14])
        r, J = orc.reproj_eval(rc, prm[o[0]:o[0] + 7], prm[o[1]:o[1] + 7], prm[o[2]:o[2] + 7], prm[o[3]:o[3] + 1],
                               prm[o[4]:o[4] + 1])
        assert np.array_equal(r, z["residuals"][i])
        assert np.array_equal(np.concatenate([x.ravel() for x in J]), z["jacobians"][i])


# ------------------------------------------------------------------- GPU: libgvx
@pytest.mark.gpu
@pytest.mark.parametrize("name", cases("klt_"))
def test_gpu_klt_golden(ctx, gvx_mod, name):
    z = load(name)
    L = int(z["levels"])
    h, w = z["I"].shape
    p = gvx_mod.KltParams.default(max_level=L)
    ctx.frame_put(31, z["I"], p)
    ctx.frame_put(32, z["J"], p)
    for k in range(L + 1):
        if f"level{k}" in z:
            assert np.array_equal(ctx.frame_level(31, k), z[f"level{k}"]), f"level {k}"
    nxt, st, err = ctx.calc_optical_flow_pyr_lk(31, 32, z["prev"], z["init"], p)
    assert np.array_equal(nxt, z["next"]) and np.array_equal(st, z["status"])
    assert np.array_equal(err[st == 1], z["err"][z["status"] == 1])
    fb = ctx.track_fb(31, 32, z["prev"], z["init"], w, h, params=p)
    for k in ("next", "back", "st_f", "st_b", "keep"):
        assert np.array_equal(fb[k], z["fb_" + k]), k
    assert np.array_equal(fb["kept_idx"], z["fb_kept"])
    # batched path (level 0 read in place)
    b = ctx.klt_fb_batch(z["I"][None], z["J"][None], z["prev"][None], z["init"][None], params=p)
    assert np.array_equal(b["next"][0], z["fb_next"]) and np.array_equal(b["back"][0], z["fb_back"])
    assert np.array_equal(b["flags"][0], z["fb_st_f"] | (z["fb_st_b"] << 1) | (z["fb_keep"] << 2))
    assert np.array_equal(b["kept"][0][:b["n_kept"][0]], z["fb_kept"])
    ctx.frame_drop(31)
    ctx.frame_drop(32)


@pytest.mark.gpu
def test_gpu_detect_golden(ctx, gvx_mod):
    z = load("detect_320x140.npz")
    ctx.frame_put(33, z["img"])
    gp = gvx_mod.DetectParams.default(max_features=int(z["max_features"]))
    c, b = ctx.detect(33, z["tracked"], z["tracked"], True, len(z["tracked"]), gp)
    assert np.array_equal(c, z["corners"])
    assert np.array_equal(b[:len(z["blocks"])], z["blocks"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", cases("preint_"))
def test_gpu_preint_golden(ctx, gvx_mod, name):
    z = load(name)
    variant = int(z["variant"])
    s = _state_fields(z)
    st = np.zeros(1, gvx_mod.STATE_DTYPE)
    for k, v in s.items():
        st[k] = v
    out, pn, pn_off = ctx.preint_integrate(variant, tuple(z["prm"]), [_imu(z)], st, z["iewn"][None])
    g = out[0]
    for k in ("p", "q", "v"):
        _close(g["delta"][k], z["delta_" + k], f"delta.{k}", 1e-10)
        _close(g["current"][k], z["current_" + k], f"current.{k}", 1e-10)
    _close(g["jacobian"].reshape(15, 15), z["jacobian"], "jacobian", 1e-10)
    _close(g["covariance"].reshape(15, 15), z["covariance"], "covariance", 1e-10)
    if variant == EARTH:
        _close(pn[:len(z["pn"])], z["pn"], "pn", 1e-10)
    res, jac = ctx.preint_factor_eval(out, pn, pn_off, z["params"], np.array([[0, 7, 16, 23]], np.int32))
    _close(res[0], z["residual"], "residual", 1e-9)
    for lo, hi in [(0, 105), (105, 240), (240, 345), (345, 480)]:
        _close(jac[0][lo:hi], z["jac"][lo:hi], f"jac[{lo}:{hi}]", 1e-9)


@pytest.mark.gpu
def test_gpu_reproj_golden(ctx, gvx_mod):
    z = load("reproj_3kf_16lm.npz")
    consts = np.ascontiguousarray(z["consts"]).view(gvx_mod.REPROJ_DTYPE).reshape(-1)
    res, jac = ctx.reproj_eval(consts, z["params"], z["offs"])
    assert np.array_equal(res, z["residuals"]) and np.array_equal(jac, z["jacobians"])


# ------------------------------------------------- preprocessing and camera ops
def _cam(mod, z):
    return mod.Camera(*[float(v) for v in z["cam"]], 1278, 1022)


@pytest.mark.parametrize("name", cases("clahe_"))
def test_oracle_clahe_golden(orc, name):
    z = load(name)
    tiles, clip = tuple(int(t) for t in z["tiles"]), float(z["clip"])
    assert np.array_equal(orc.clahe_luts(z["img"], clip, tiles), z["luts"])
    assert np.array_equal(orc.clahe(z["img"], clip, tiles), z["out"])
    assert orc.hist_mean(z["img"]) == float(z["hist_mean"])


def test_oracle_camera_golden(orc):
    z = load("camera_kaist_n200.npz")
    c = _cam(orc, z)
    assert np.array_equal(orc.undistort_points(c, z["p"]), z["undist"])
    assert np.array_equal(orc.distort_points(c, z["p"]), z["dist"])
    assert np.array_equal(orc.predict_rotated(c, z["R"], z["p"]), z["pred"])
    assert np.array_equal(orc.project_points(c, z["R0"], z["t"], z["pw"]), z["proj"])
    assert np.array_equal(orc.point_velocity(c, z["p"], z["q"], 0.05), z["vel"])
    assert np.array_equal(orc.keypoint_parallax(c, z["R0"], z["R1"], z["p"], z["q"]), z["parallax"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", cases("clahe_"))
def test_gpu_clahe_golden(ctx, gvx_mod, name):
    z = load(name)
    tiles = tuple(int(t) for t in z["tiles"])
    p = gvx_mod.ClaheParams.default(clip_limit=float(z["clip"]), tiles_x=tiles[0], tiles_y=tiles[1])
    out, m = ctx.clahe(z["img"], p, hist_mean=True)
    assert np.array_equal(out, z["out"]) and m == float(z["hist_mean"])


@pytest.mark.gpu
def test_gpu_camera_golden(ctx, gvx_mod):
    z = load("camera_kaist_n200.npz")
    c = _cam(gvx_mod, z)
    assert np.array_equal(ctx.undistort_points(c, z["p"]), z["undist"])
    assert np.array_equal(ctx.distort_points(c, z["p"]), z["dist"])
    assert np.array_equal(ctx.predict_rotated(c, z["R"], z["p"]), z["pred"])
    assert np.array_equal(ctx.project_points(c, z["R0"], z["t"], z["pw"]), z["proj"])
    assert np.array_equal(ctx.point_velocity(c, z["p"], z["q"], 0.05), z["vel"])
    assert np.array_equal(ctx.keypoint_parallax(c, z["R0"], z["R1"], z["p"], z["q"]), z["parallax"])
