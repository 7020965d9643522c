"""The C++ host mirror (ic-gvins_amd/host/include/gvx/gvx.hpp) of the reference
interfaces -- cv::calcOpticalFlowPyrLK, the fused FB tracking + reduceVector,
featuresDetection, PreintegrationBase (addNewImu / reintegration / getters),
PreintegrationFactor / ReprojectionFactor::Evaluate -- compiled with g++ against
libgvx.so (tests/host/test_host.cpp).  CPU: it builds, links and fails loudly
without a device.  GPU: its outputs equal the oracle's (bit-exact KLT /
detection / reprojection, 1e-10 / 1e-9 for the fp64 preintegration path)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NORMAL, EARTH = 0, 2


@pytest.fixture(scope="module")
def host_bin(tmp_path_factory, gvx_mod):
    out = str(tmp_path_factory.mktemp("host") / "test_host")
    libdir = os.path.dirname(gvx_mod.LIB_PATH)
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(ROOT, "ic-gvins_amd", "host", "include"),
           os.path.join(ROOT, "tests", "host", "test_host.cpp"), "-o", out, "-L", libdir, "-lgvx",
           f"-Wl,-rpath,{libdir}", "-Wl,-rpath-link,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


def test_host_mirror_builds_and_fails_loudly_without_device(host_bin):
    import torch
    r = subprocess.run([host_bin, "nodev"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    if not torch.cuda.is_available():
        assert r.stdout.startswith("ERROR -2"), r.stdout


def _close(g, o, what, rtol):
    g, o = np.asarray(g, np.float64), np.asarray(o, np.float64)
    scale = max(np.abs(o).max(), 1e-300)
    assert np.abs(g - o).max() <= rtol * scale, f"{what}: {np.abs(g - o).max():.3e} vs scale {scale:.3e}"


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [NORMAL, EARTH])
def test_host_mirror_matches_oracle(host_bin, orc, tmp_path, variant):
    from gvx import synth, synth_ba
    d = str(tmp_path)
    w, h, n = 640, 280, 96
    I, J, prev, init, _ = synth.make_pair(w, h, n, seed=77 + variant)
    rng = np.random.default_rng(5 + variant)
    imu = synth_ba.make_imu_segment(rng, 60)
    s = synth_ba.random_state(rng)
    st = np.r_[s["time"], s["p"], s["q"], s["v"], s["bg"], s["ba"]].astype(np.float64)
    prm = np.array(synth_ba.imu_params(), np.float64)
    np.array([w, h, n, variant], np.int32).tofile(f"{d}/meta.bin")
    I.tofile(f"{d}/I.bin"), J.tofile(f"{d}/J.bin")
    prev.astype(np.float32).tofile(f"{d}/prev.bin"), init.astype(np.float32).tofile(f"{d}/init.bin")
    imu.tofile(f"{d}/imu.bin"), st.tofile(f"{d}/state.bin"), prm.tofile(f"{d}/prm.bin")
    iewn = orc.earth_iewn(np.zeros(3), s["p"])  # IntegrationParameters::station defaults to 0
    seg = orc.PreintSeg(variant, orc.imu_params(*prm), imu,
                        orc.make_state(float(s["time"]), s["p"], s["q"], s["v"], s["bg"], s["ba"]), iewn)
    c = seg.current()
    blocks = (np.r_[s["p"], s["q"]], np.r_[s["v"], s["bg"], s["ba"]] + 1e-4,
              np.r_[c["p"] + 0.01, c["q"]], np.r_[c["v"], c["bg"], c["ba"]] - 1e-4)
    np.concatenate(blocks).tofile(f"{d}/fparams.bin")
    prob = synth_ba.make_ba_problem(n_kf=3, n_lm=4)
    rc, o = prob["consts"][0], prob["offs"][0]
    rconst = np.r_[rc["pts0"], rc["pts1"], rc["vel0"], rc["vel1"], rc["td0"], rc["td1"], rc["std"]]
    rconst.astype(np.float64).tofile(f"{d}/rconst.bin")
    pr = prob["params"]
    rblocks = [pr[o[0]:o[0] + 7], pr[o[1]:o[1] + 7], pr[o[2]:o[2] + 7], pr[o[3]:o[3] + 1], pr[o[4]:o[4] + 1]]
    np.concatenate(rblocks).tofile(f"{d}/rparams.bin")

    cam = (787.1611861559479, 787.3928431375225, 664.4061078354368, 519.5129292754456, 0.0,
           -0.0917403092279957, 0.08134715036932794, 0.00017620136958692255, 0.00016737385248865412, 0.0)
    np.array(cam, np.float64).tofile(f"{d}/cam.bin")
    a, b = 0.02 + 0.01 * variant, 0.3
    Rc = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
    R0 = np.array([[np.cos(b), -np.sin(b), 0], [np.sin(b), np.cos(b), 0], [0, 0, 1]])
    np.concatenate([Rc.ravel(), R0.ravel(), (Rc @ R0).ravel()]).tofile(f"{d}/rot.bin")

    r = subprocess.run([host_bin, "run", d], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr

    rd = lambda name, dt: np.fromfile(f"{d}/{name}", dt)  # noqa: E731
    o_next, o_st, o_err = orc.calc_optical_flow_pyr_lk(I, J, prev, init)
    assert np.array_equal(rd("lk_next.bin", np.float32).reshape(-1, 2), o_next)
    assert np.array_equal(rd("lk_status.bin", np.uint8), o_st)
    assert np.array_equal(rd("lk_err.bin", np.float32)[o_st == 1], o_err[o_st == 1])
    fb = orc.klt_fb(I, J, prev, init, w, h, reuse_pyramids=True)
    assert np.array_equal(rd("fb_next.bin", np.float32).reshape(-1, 2), fb["next"])
    assert np.array_equal(rd("fb_back.bin", np.float32).reshape(-1, 2), fb["back"])
    assert np.array_equal(rd("fb_keep.bin", np.uint8), fb["keep"])
    assert np.array_equal(rd("fb_kept.bin", np.int32), fb["kept_idx"])
    assert np.array_equal(rd("fb_reduced.bin", np.float32).reshape(-1, 2), fb["next"][fb["kept_idx"]])
    det, _ = orc.features_detection(I, None, None, False, 0, orc.DetectParams.default())
    assert np.array_equal(rd("det.bin", np.float32).reshape(-1, 2), det)
    assert np.array_equal(rd("clahe.bin", np.uint8).reshape(h, w), orc.clahe(I))
    assert rd("hist_mean.bin", np.float64)[0] == orc.hist_mean(I)
    oc = orc.Camera(*cam, w, h)
    assert np.array_equal(rd("cam_undist.bin", np.float32).reshape(-1, 2), orc.undistort_points(oc, prev))
    assert np.array_equal(rd("cam_dist.bin", np.float32).reshape(-1, 2), orc.distort_points(oc, prev))
    assert np.array_equal(rd("cam_pred.bin", np.float32).reshape(-1, 2), orc.predict_rotated(oc, Rc, prev))
    assert np.array_equal(rd("cam_vel.bin", np.float64).reshape(-1, 2), orc.point_velocity(oc, prev, init, 0.05))
    assert np.array_equal(rd("cam_par.bin", np.float64), orc.keypoint_parallax(oc, R0, Rc @ R0, prev, init))

    ps = rd("pre_state.bin", np.float64)
    dlt, cur = seg.delta(), seg.current()
    for k, (lo, hi) in (("p", (1, 4)), ("q", (4, 8)), ("v", (8, 11))):
        _close(ps[lo:hi], dlt[k], f"delta.{k}", 1e-10)
        _close(ps[17 + lo:17 + hi], cur[k], f"current.{k}", 1e-10)
    assert ps[34] == pytest.approx(seg.s.delta_time, rel=1e-15)
    if variant == EARTH:
        _close(rd("pre_pn.bin", np.float64).reshape(-1, 4), seg.pn, "pn", 1e-10)
    pf = rd("pf.bin", np.float64)
    res, Jo = seg.evaluate(*blocks)
    _close(pf[:15], res, "factor residual", 1e-9)
    oj = np.concatenate([x.ravel() for x in Jo])
    for b, (lo, hi) in enumerate([(0, 105), (105, 240), (240, 345), (345, 480)]):
        _close(pf[15 + lo:15 + hi], oj[lo:hi], f"factor J{b}", 1e-9)
    bg2, ba2 = s["bg"].copy(), s["ba"].copy()
    bg2[0] += 1e-3
    ba2[2] -= 2e-3
    seg2 = orc.PreintSeg(variant, orc.imu_params(*prm), imu,
                         orc.make_state(float(s["time"]), s["p"], s["q"], s["v"], bg2, ba2), iewn)
    ps2 = rd("pre_state2.bin", np.float64)
    for k, (lo, hi) in (("p", (1, 4)), ("q", (4, 8)), ("v", (8, 11))):
        _close(ps2[lo:hi], seg2.delta()[k], f"reintegrated delta.{k}", 1e-10)
    # MISC::redoInsMechanization on the deque window + pop_front, getImuSeriesFromTo, GnssFactor
    g = prm[5]
    iewn_ins = (1e-5, 2e-5, 6e-5) if variant == EARTH else (0.0, 0.0, 0.0)
    ocfg = orc.InsConfig.make(variant == EARTH, (0, 0, g), iewn_ins)
    states = np.array([s] * len(imu))
    upd = orc.make_state(float(imu[20]["time"]) + 0.0021, s["p"], s["q"], s["v"], s["bg"], s["ba"])
    idx = orc.redo_ins_mechanization(ocfg, upd, imu, states)
    assert idx == 21
    kept = states[idx - 8:]
    got = rd("ins_redo.bin", np.float64)
    assert int(got[0]) == len(kept)
    got = got[1:].reshape(-1, 17)
    ref = np.stack([np.r_[k["time"], k["p"], k["q"], k["v"], k["bg"], k["ba"]] for k in kept])
    assert np.array_equal(got[:, 0], ref[:, 0]) and np.array_equal(got[:, 11:], ref[:, 11:])
    _close(got[:, 1:11], ref[:, 1:11], "redoInsMechanization p/q/v", 1e-10)
    ser = orc.imu_series_from_to(imu[idx - 8:], float(imu[25]["time"]) + 0.001, float(imu[40]["time"]) + 0.003)
    assert np.array_equal(rd("ins_series.bin", np.float64), ser.view(np.float64).ravel())
    gr, gj = orc.small_factor_eval(0, np.r_[1.0, 2.0, 3.0, 0.02, 0.03, 0.05, 0.1, -0.2, 0.3], blocks[0], [0])
    _close(rd("gnss.bin", np.float64), gr[0], "GnssFactor residual", 1e-12)
    _close(rd("gnss_jac.bin", np.float64), gj[0], "GnssFactor jacobian", 1e-12)
    rf = rd("rf.bin", np.float64)
    rcc = orc.reproj_const(rc["pts0"], rc["pts1"], rc["vel0"], rc["vel1"], rc["td0"], rc["td1"], rc["std"])
    rr, rj = orc.reproj_eval(rcc, *rblocks)
    assert np.array_equal(rf[:2], rr)
    assert np.array_equal(rf[2:], np.concatenate([x.ravel() for x in rj]))


@pytest.fixture(scope="module")
def marg_bin(tmp_path_factory, gvx_mod):
    out = str(tmp_path_factory.mktemp("host") / "test_marg_host")
    libdir = os.path.dirname(gvx_mod.LIB_PATH)
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(ROOT, "ic-gvins_amd", "host", "include"),
           os.path.join(ROOT, "tests", "host", "test_marg_host.cpp"), "-o", out, "-L", libdir, "-lgvx",
           f"-Wl,-rpath,{libdir}", "-Wl,-rpath-link,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


def _marg_files(d, orc):
    """The configs[3]-shaped problem (synth_ba.make_marg_problem, small) as
    replayable residual blocks for the C++ mirror."""
    from gvx import synth_ba
    p = synth_ba.make_marg_problem(orc.FactorEvaluator(), n_kf=4, n_lm=12)
    nb = len(p["size"])
    rng = np.random.default_rng(2)
    vals = [rng.normal(size=int(s)) for s in p["size"]]
    np.asarray(p["size"], np.int32).tofile(f"{d}/bsize.bin")
    np.concatenate(vals).tofile(f"{d}/bval.bin")
    meta, blk, marg, data = [], [], [], []
    for f in range(len(p["nres"])):
        bl = p["blk"][p["blk_off"][f]:p["blk_off"][f + 1]]
        mg = [k for k, b in enumerate(bl) if p["index"][b] < p["m"]]
        meta += [int(p["nres"][f]), len(bl), len(mg)]
        blk += list(bl)
        marg += mg
        n = int(p["nres"][f]) * (1 + int(p["size"][bl].sum()))
        data.append(p["data"][p["res_off"][f]:p["res_off"][f] + n])
    np.asarray(meta, np.int32).tofile(f"{d}/fmeta.bin")
    np.asarray(blk, np.int32).tofile(f"{d}/fblk.bin")
    np.asarray(marg, np.int32).tofile(f"{d}/fmarg.bin")
    np.concatenate(data).tofile(f"{d}/fdata.bin")
    return p, nb


def test_marg_mirror_fails_loudly_without_device(marg_bin, orc, tmp_path):
    import torch
    _marg_files(str(tmp_path), orc)
    r = subprocess.run([marg_bin, str(tmp_path), "nodev"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    if not torch.cuda.is_available():
        assert r.stdout.startswith("ERROR -2"), r.stdout


@pytest.mark.gpu
def test_marg_mirror_matches_oracle(marg_bin, orc, tmp_path):
    """The mirror's block order comes from the reference's unordered_map walk;
    given that order, its device J0 / e0 equal the restatement's bit for bit, and
    the next MarginalizationFactor at the linearisation point returns e0."""
    d = str(tmp_path)
    p, nb = _marg_files(d, orc)
    r = subprocess.run([marg_bin, d, "exact"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
    index = np.fromfile(f"{d}/index.bin", np.int32)
    marg = set(np.nonzero(p["index"] < p["m"])[0])
    m = int(sum(6 if p["size"][b] == 7 else p["size"][b] for b in marg))
    assert all(index[b] < m for b in marg) and all(index[b] >= m for b in range(nb) if b not in marg)
    q = dict(p, index=index)
    H0, b0 = orc.marg_construct(q)
    Hp, bp, _ = orc.marg_schur(H0, b0, m)
    J0, e0, _, _ = orc.marg_linearize(Hp, bp)
    r_ = p["L"] - m
    assert np.array_equal(np.fromfile(f"{d}/J0.bin").reshape(r_, r_).T, J0)
    assert np.array_equal(np.fromfile(f"{d}/e0.bin"), e0)
    res = np.fromfile(f"{d}/res.bin")
    np.testing.assert_allclose(res, e0, rtol=0, atol=1e-14 * np.abs(J0).sum(1).max())


@pytest.mark.gpu
def test_marg_mirror_fast_solver(marg_bin, orc, tmp_path):
    """The mirror with the default FAST solver (device Cholesky): J0 / e0 are a
    different factorisation of the same prior, so they are checked by what the
    next window uses -- J0^T J0 = Hp and J0^T e0 = -bp (marginalization_info.h:153-167)
    -- and the next MarginalizationFactor at the linearisation point returns e0."""
    d = str(tmp_path)
    p, nb = _marg_files(d, orc)
    r = subprocess.run([marg_bin, d], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
    index = np.fromfile(f"{d}/index.bin", np.int32)
    marg = set(np.nonzero(p["index"] < p["m"])[0])
    m = int(sum(6 if p["size"][b] == 7 else p["size"][b] for b in marg))
    H0, b0 = orc.marg_construct(dict(p, index=index))
    Hp, bp, _ = orc.marg_schur(H0, b0, m)
    r_ = p["L"] - m
    J0 = np.fromfile(f"{d}/J0.bin").reshape(r_, r_).T
    e0 = np.fromfile(f"{d}/e0.bin")
    scale = np.abs(Hp).max()
    np.testing.assert_allclose(J0.T @ J0, Hp, rtol=0, atol=1e-9 * scale)
    np.testing.assert_allclose(J0.T @ e0, -bp, rtol=0, atol=1e-9 * max(np.abs(bp).max(), 1.0))
    res = np.fromfile(f"{d}/res.bin")
    np.testing.assert_allclose(res, e0, rtol=0, atol=1e-14 * np.abs(J0).sum(1).max())
