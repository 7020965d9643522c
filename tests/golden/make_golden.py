#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the CPU restatement
(oracle/, test infrastructure).

The reference holds no fixtures or tests for this path, and its arithmetic lives in
un-vendored OpenCV / Eigen that cannot be built or imported here (SURVEY.md
8c), so these vectors are *regression pins* of the restatement (parity
unpinned against OpenCV itself).  They are small (about
200 KB total), numeric-only .npz files (np.load(..., allow_pickle=False)), and
tests/test_golden.py checks both the oracle (CPU) and libgvx (GPU) against them.

    python tests/golden/make_golden.py [name.npz ...]   # rewrites tests/golden/*.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "ic-gvins_amd"))

import oracle as orc  # noqa: E402
from gvx import synth, synth_ba  # noqa: E402

NORMAL, EARTH = 0, 2


def klt_case(name, w, h, n, levels, seed):
    I, J, prev, init, _ = synth.make_pair(w, h, n, seed)
    p = orc.KltParams.default(max_level=levels)
    nxt, st, err = orc.calc_optical_flow_pyr_lk(I, J, prev, init, p)
    fb = orc.klt_fb(I, J, prev, init, w, h, params=p, reuse_pyramids=True)
    pyr = orc.build_pyramid(I, levels)
    lv = {f"level{k}": v for k, v in enumerate(pyr)}
    np.savez_compressed(os.path.join(HERE, name), I=I, J=J, prev=prev, init=init, levels=np.int32(levels),
                        next=nxt, status=st, err=err, fb_next=fb["next"], fb_back=fb["back"], fb_st_f=fb["st_f"],
                        fb_st_b=fb["st_b"], fb_keep=fb["keep"], fb_kept=fb["kept_idx"].astype(np.int32), **lv)


def detect_case(name, w, h, seed, n_tracked):
    rng = np.random.default_rng(seed)
    img = synth.make_image(w, h, rng)
    pts = np.c_[rng.uniform(0, w, n_tracked), rng.uniform(0, h, n_tracked)].astype(np.float32)
    prm = orc.DetectParams.default(max_features=80)
    corners, blocks = orc.features_detection(img, pts, pts, True, n_tracked, prm)
    np.savez_compressed(os.path.join(HERE, name), img=img, tracked=pts, max_features=np.int32(80),
                        corners=corners, blocks=np.asarray(blocks, np.int32))


def preint_case(name, variant, m, seed):
    rng = np.random.default_rng(seed)
    imu = synth_ba.make_imu_segment(rng, m)
    s = synth_ba.random_state(rng)
    prm = np.array(synth_ba.imu_params(), np.float64)
    iewn = np.asarray(orc.earth_iewn(np.zeros(3), s["p"]), np.float64)
    st = orc.make_state(float(s["time"]), s["p"], s["q"], s["v"], s["bg"], s["ba"])
    seg = orc.PreintSeg(variant, orc.imu_params(*prm), imu, st, iewn)
    d, c = seg.delta(), seg.current()
    # factor evaluation near the integrated state
    blocks = (np.r_[s["p"], s["q"]], np.r_[s["v"], s["bg"], s["ba"]] + 1e-4,
              np.r_[c["p"] + 0.01, c["q"]], np.r_[c["v"], c["bg"], c["ba"]] - 1e-4)
    res, J = seg.evaluate(*blocks)
    state0 = np.r_[s["time"], s["p"], s["q"], s["v"], s["bg"], s["ba"]].astype(np.float64)
    np.savez_compressed(os.path.join(HERE, name), variant=np.int32(variant), imu=imu.view(np.float64).reshape(m, 9),
                        state0=state0, prm=prm, iewn=iewn, delta_time=np.float64(seg.s.delta_time),
                        delta_p=d["p"], delta_q=d["q"], delta_v=d["v"], current_p=c["p"], current_q=c["q"],
                        current_v=c["v"], jacobian=seg.jacobian, covariance=seg.covariance,
                        pn=seg.pn if variant == EARTH else np.zeros((0, 4)), params=np.concatenate(blocks),
                        residual=res, jac=np.concatenate([x.ravel() for x in J]))


def reproj_case(name, n_kf, n_lm):
    prob = synth_ba.make_ba_problem(n_kf=n_kf, n_lm=n_lm)
    cs, prm, offs = prob["consts"], prob["params"], prob["offs"]
    res, jac = [], []
    for i in range(len(cs)):
        c, o = cs[i], offs[i]
        rc = orc.reproj_const(c["pts0"], c["pts1"], c["vel0"], c["vel1"], c["td0"], c["td1"], c["std"])
        r, J = orc.reproj_eval(rc, prm[o[0]:o[0] + 7], prm[o[1]:o[1] + 7], prm[o[2]:o[2] + 7],
                               prm[o[3]:o[3] + 1], prm[o[4]:o[4] + 1])
        res.append(r)
        jac.append(np.concatenate([x.ravel() for x in J]))
    consts = np.stack([np.r_[c["pts0"], c["pts1"], c["vel0"], c["vel1"], c["td0"], c["td1"], c["std"]]
                       for c in cs]).astype(np.float64)
    np.savez_compressed(os.path.join(HERE, name), consts=consts, params=prm, offs=offs.astype(np.int32),
                        residuals=np.array(res), jacobians=np.array(jac))


def clahe_case(name, w, h, tiles, clip, seed):
    img = synth.make_image(w, h, np.random.default_rng(seed))
    np.savez_compressed(os.path.join(HERE, name), img=img, tiles=np.int32(tiles), clip=np.float64(clip),
                        luts=orc.clahe_luts(img, clip, tiles), out=orc.clahe(img, clip, tiles),
                        hist_mean=np.float64(orc.hist_mean(img)))


# config/gvins.yaml:65-73 (k3 = 0 for the 4-term distortion, camera.cc:62-64)
KAIST_CAM = (787.1611861559479, 787.3928431375225, 664.4061078354368, 519.5129292754456, 0.0,
             -0.0917403092279957, 0.08134715036932794, 0.00017620136958692255, 0.00016737385248865412, 0.0)


def camera_case(name, n, seed):
    rng = np.random.default_rng(seed)
    cam = orc.Camera(*KAIST_CAM, 1278, 1022)
    p = np.c_[rng.uniform(-20, 1298, n), rng.uniform(-20, 1042, n)].astype(np.float32)
    q = (p + rng.uniform(-4, 4, (n, 2))).astype(np.float32)
    a = 0.03
    R = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
    R0 = np.array([[np.cos(0.4), -np.sin(0.4), 0], [np.sin(0.4), np.cos(0.4), 0], [0, 0, 1]])
    R1 = R @ R0
    t = np.array([0.3, -1.2, 2.0])
    pc = np.c_[rng.uniform(-8, 8, n), rng.uniform(-4, 4, n), rng.uniform(3, 60, n)]
    pw = pc @ R0.T + t
    np.savez_compressed(os.path.join(HERE, name), cam=np.array(KAIST_CAM), p=p, q=q, R=R, R0=R0, R1=R1, t=t, pw=pw,
                        undist=orc.undistort_points(cam, p), dist=orc.distort_points(cam, p),
                        pred=orc.predict_rotated(cam, R, p), proj=orc.project_points(cam, R0, t, pw),
                        vel=orc.point_velocity(cam, p, q, 0.05), parallax=orc.keypoint_parallax(cam, R0, R1, p, q))


CASES = {
    "klt_160x70_n32_L3.npz": lambda n: klt_case(n, 160, 70, 32, 3, 1),
    "klt_320x140_n64_L3.npz": lambda n: klt_case(n, 320, 140, 64, 3, 2),
    "klt_333x97_n40_L2.npz": lambda n: klt_case(n, 333, 97, 40, 2, 3),
    "detect_320x140.npz": lambda n: detect_case(n, 320, 140, 11, 12),
    "preint_normal_m20.npz": lambda n: preint_case(n, NORMAL, 20, 41),
    "preint_earth_m20.npz": lambda n: preint_case(n, EARTH, 20, 42),
    "preint_earth_m100.npz": lambda n: preint_case(n, EARTH, 100, 43),
    "reproj_3kf_16lm.npz": lambda n: reproj_case(n, 3, 16),
    "clahe_320x140_t21.npz": lambda n: clahe_case(n, 320, 140, (21, 21), 3.0, 51),
    "clahe_215x147_t8x6.npz": lambda n: clahe_case(n, 215, 147, (8, 6), 2.0, 52),
    "camera_kaist_n200.npz": lambda n: camera_case(n, 200, 61),
}

if __name__ == "__main__":
    # python make_golden.py [case ...]: only the named fixtures (default: all)
    for name in (sys.argv[1:] or list(CASES)):
        CASES[name](name)
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
