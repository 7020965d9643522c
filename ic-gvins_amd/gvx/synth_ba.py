"""Synthetic IMU segments and sliding-window BA problems.

Noise / extrinsic / camera values come from the reference's config
(/root/reference/config/gvins.yaml:26-31, :64-79) converted the way the GVINS
ctor does (ic_gvins/ic_gvins/ic_gvins.cc:103-110, :157):
  gyr_arw = arw * D2R / 60, acc_vrw = vrw / 60, gyr_bias_std = gbstd * D2R / 3600,
  acc_bias_std = abstd * 1e-5, corr_time = corrtime * 3600, gravity = NORMAL_GRAVITY.
Data is synthetic (no bags offline): a 5 m/s trajectory, 0.5 s keyframes, 200 Hz IMU.
"""
from __future__ import annotations

import numpy as np

D2R = np.pi / 180.0
NORMAL_GRAVITY = 9.80  # GVINS::NORMAL_GRAVITY, ic_gvins/ic_gvins/ic_gvins.h:120
IMU_DTYPE = np.dtype([("time", "f8"), ("dt", "f8"), ("dtheta", "f8", 3), ("dvel", "f8", 3),
                      ("odovel", "f8")])
STATE_DTYPE = np.dtype([("time", "f8"), ("p", "f8", 3), ("q", "f8", 4), ("v", "f8", 3), ("bg", "f8", 3),
                        ("ba", "f8", 3)])
REPROJ_DTYPE = np.dtype([("pts0", "f8", 3), ("pts1", "f8", 3), ("vel0", "f8", 3), ("vel1", "f8", 3),
                         ("td0", "f8"), ("td1", "f8"), ("std", "f8")])

# config/gvins.yaml
CFG_ARW, CFG_VRW, CFG_GBSTD, CFG_ABSTD, CFG_CORRTIME = 0.1, 0.1, 50.0, 50.0, 1.0
FX = 787.1611861559479
Q_B_C = np.array([0.497766, 0.502679, 0.501396, 0.498141])  # x y z w
T_B_C = np.array([0.074, -0.030, 0.128])
REPROJ_STD_PX = 1.5


def imu_params():
    """(acc_vrw, gyr_arw, gyr_bias_std, acc_bias_std, corr_time, gravity)"""
    return (CFG_VRW / 60.0, CFG_ARW * D2R / 60.0, CFG_GBSTD * D2R / 3600.0, CFG_ABSTD * 1.0e-5,
            CFG_CORRTIME * 3600.0, NORMAL_GRAVITY)


def quat_mul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by + ay * bw + az * bx - ax * bz,
                     aw * bz + az * bw + ax * by - ay * bx, aw * bw - ax * bx - ay * by - az * bz])


def quat_from_rotvec(r):
    a = np.linalg.norm(r)
    if a == 0:
        return np.array([0.0, 0.0, 0.0, 1.0])
    s = np.sin(a / 2) / a
    return np.array([r[0] * s, r[1] * s, r[2] * s, np.cos(a / 2)])


def quat_to_rot(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def make_imu_segment(rng, m=100, rate=200.0, t0=0.0, speed=5.0, noisy=True):
    """m IMU increments (the reference's vector<IMU> from getImuSeriesFromTo):
    smooth body rates/accelerations around a 5 m/s forward motion."""
    dt = 1.0 / rate
    imu = np.zeros(m, IMU_DTYPE)
    w0 = rng.normal(0, 0.05, 3)
    a0 = rng.normal(0, 0.3, 3) + np.array([0.0, 0.0, -NORMAL_GRAVITY])
    ph = rng.uniform(0, 2 * np.pi, 3)
    arw, vrw = CFG_ARW * D2R / 60.0, CFG_VRW / 60.0
    for k in range(m):
        t = t0 + k * dt
        w = w0 + 0.02 * np.sin(2 * np.pi * 0.5 * t + ph)
        a = a0 + 0.2 * np.cos(2 * np.pi * 0.7 * t + ph)
        imu[k]["time"] = t
        imu[k]["dt"] = dt if k > 0 else dt
        imu[k]["dtheta"] = w * dt + (rng.normal(0, arw * np.sqrt(dt), 3) if noisy else 0)
        imu[k]["dvel"] = a * dt + (rng.normal(0, vrw * np.sqrt(dt), 3) if noisy else 0)
    return imu


def random_state(rng, t=0.0):
    s = np.zeros((), STATE_DTYPE)
    s["time"] = t
    s["p"] = rng.normal(0, 10, 3)
    q = quat_from_rotvec(rng.normal(0, 0.3, 3))
    s["q"] = q / np.linalg.norm(q)
    s["v"] = np.array([5.0, 0, 0]) + rng.normal(0, 0.1, 3)
    s["bg"] = rng.normal(0, CFG_GBSTD * D2R / 3600.0, 3)
    s["ba"] = rng.normal(0, CFG_ABSTD * 1e-5, 3)
    return s


def make_ba_problem(seed=20261015, n_kf=10, n_lm=200, dt_kf=0.5):
    """Sliding-window BA instance (config 4): keyframe poses (p, q xyzw) of the IMU
    body, landmarks referenced in their first keyframe and observed in all later
    ones -> n_lm * (n_kf - 1) reprojection factors."""
    rng = np.random.default_rng(seed)
    R_bc = quat_to_rot(Q_B_C)
    poses = np.zeros((n_kf, 7))
    for k in range(n_kf):
        poses[k, :3] = [5.0 * dt_kf * k, 0.2 * np.sin(k), 0.05 * k]
        q = quat_from_rotvec(np.array([0.01 * k, -0.02 * k, 0.03 * np.sin(k)]))
        poses[k, 3:] = q / np.linalg.norm(q)
    ext = np.concatenate([T_B_C, Q_B_C / np.linalg.norm(Q_B_C)])
    consts = np.zeros((n_lm * (n_kf - 1),), REPROJ_DTYPE)
    offs = []
    invdepth = np.zeros(n_lm)
    std = REPROJ_STD_PX / FX
    f = 0
    for j in range(n_lm):
        # landmark in the first keyframe's camera: depth 5..50 m, inside the FOV
        d = rng.uniform(5, 50)
        uv = rng.uniform(-0.5, 0.5, 2)
        pc0 = np.array([uv[0] * d, uv[1] * d, d])
        invdepth[j] = 1.0 / d
        Rb0 = quat_to_rot(poses[0, 3:])
        pw = Rb0 @ (R_bc @ pc0 + T_B_C) + poses[0, :3]
        vel0 = rng.normal(0, 0.05, 3)
        vel0[2] = 0
        for k in range(1, n_kf):
            Rbk = quat_to_rot(poses[k, 3:])
            pb = Rbk.T @ (pw - poses[k, :3])
            pc = R_bc.T @ (pb - T_B_C)
            pts1 = np.array([pc[0] / pc[2], pc[1] / pc[2], 1.0]) + np.r_[rng.normal(0, std, 2), 0]
            vel1 = rng.normal(0, 0.05, 3)
            vel1[2] = 0
            consts[f] = (np.array([uv[0], uv[1], 1.0]), pts1, vel0, vel1, 0.0, 0.0, std)
            offs.append((0, k, 0, j, 0))
            f += 1
    # packed parameter array: poses | ext | invdepths | td
    params = np.concatenate([poses.reshape(-1), ext, invdepth, [0.0]])
    o_pose, o_ext, o_id, o_td = 0, 7 * n_kf, 7 * n_kf + 7, 7 * n_kf + 7 + n_lm
    offs = np.array([[o_pose + 7 * a, o_pose + 7 * b, o_ext, o_id + j, o_td] for a, b, _, j, _ in offs],
                    np.int32)
    return dict(params=params, offs=offs, consts=consts, poses=poses, ext=ext, invdepth=invdepth)
