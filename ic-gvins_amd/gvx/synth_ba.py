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


def _pose_block_values(rng, n):
    q = np.array([quat_from_rotvec(rng.normal(0, 0.3, 3)) for _ in range(n)])
    return np.concatenate([rng.normal(0, 10, (n, 3)), q / np.linalg.norm(q, axis=1, keepdims=True)], axis=1)


def make_marg_problem(ev, seed=20261015, n_kf=10, n_lm=200, n_prior_kf=None, gnss=True, huber=None):
    """MarginalizationInfo input when the oldest keyframe leaves the window, in
    the order IC-GVINS adds the residual blocks (ic_gvins.cc:1514-1644):
      1. the previous MarginalizationFactor over pose/mix of keyframes
         0..n_prior_kf-1 + extrinsic + td (marginalized: pose0, mix0),
      2. a GnssFactor on pose0,
      3. the PreintegrationFactor 0 -> 1 (Earth variant, M = 100; marginalized: pose0, mix0),
      4. the ReprojectionFactors of the landmarks referenced in keyframe 0, observed in
         keyframes 1..n_kf-1 (the configs[3] window; marginalized: pose0, invdepth),
    each evaluated by `ev` (an object with reproj / preint / gnss / marg methods:
    the oracle in tests, the device in the benchmark).  huber: HuberLoss parameter
    for the reprojection blocks (the reference passes nullptr, i.e. None).
    Marginalized blocks get the first local indices (pose0, mix0, invdepths), the
    remained ones follow in block order.  Returns the dict gvx.Context.marginalize
    and oracle.marg_construct take."""
    rng = np.random.default_rng(seed)
    n_prior_kf = n_kf if n_prior_kf is None else n_prior_kf
    ba = make_ba_problem(seed, n_kf, n_lm)
    poses, ext, invd = ba["poses"], ba["ext"], ba["invdepth"]
    mixes = np.concatenate([np.tile([5.0, 0.0, 0.0], (n_kf, 1)) + rng.normal(0, 0.1, (n_kf, 3)),
                            rng.normal(0, CFG_GBSTD * D2R / 3600.0, (n_kf, 3)),
                            rng.normal(0, CFG_ABSTD * 1e-5, (n_kf, 3))], axis=1)
    # block table: pose k, mix k, ext, td, invdepth j
    names, size, vals = [], [], []
    for k in range(n_kf):
        names += [f"pose{k}", f"mix{k}"]
        size += [7, 9]
        vals += [poses[k], mixes[k]]
    names += ["ext", "td"]
    size += [7, 1]
    vals += [ext, np.zeros(1)]
    for j in range(n_lm):
        names.append(f"invdepth{j}")
        size.append(1)
        vals.append(invd[j:j + 1])
    bid = {n: i for i, n in enumerate(names)}
    facs = []  # (blocks, residuals, jacobian)
    # 1. previous marginalisation factor
    pb = [bid[f"{t}{k}"] for k in range(n_prior_kf) for t in ("pose", "mix")] + [bid["ext"], bid["td"]]
    psz = [size[b] for b in pb]
    ploc = [6 if s == 7 else s for s in psz]
    r_prev = int(sum(ploc))
    pidx = np.concatenate([[0], np.cumsum(ploc)[:-1]]).astype(np.int32)
    pxo = np.concatenate([[0], np.cumsum(psz)[:-1]]).astype(np.int32)
    x = np.concatenate([vals[b] for b in pb])
    x0 = x.copy()
    for b, o in zip(pb, pxo):
        if size[b] == 7:
            x0[o:o + 3] += rng.normal(0, 0.01, 3)
            q = quat_mul(x0[o + 3:o + 7], quat_from_rotvec(rng.normal(0, 1e-3, 3)))
            x0[o + 3:o + 7] = q / np.linalg.norm(q)
        else:
            x0[o:o + size[b]] += rng.normal(0, 1e-3, size[b])
    # J0 of a previous Hp: information from 1e0 to 1e8 across the remained states
    A = rng.normal(size=(r_prev, r_prev))
    H = A @ A.T / r_prev + np.eye(r_prev)
    D = np.diag(10 ** rng.uniform(0, 4, r_prev))
    J0 = np.linalg.cholesky(D @ H @ D).T
    e0 = rng.normal(0, 1, r_prev)
    res, jac = ev.marg(psz, pidx, pxo, x0, x, J0, e0)
    facs.append((pb, res, jac))
    # 2. GNSS on pose0
    if gnss:
        gc = np.concatenate([poses[0, :3] + rng.normal(0, 0.05, 3), [0.02, 0.02, 0.05], [0.1, -0.2, 0.3]])
        res, jac = ev.gnss(gc, poses[0])
        facs.append(([bid["pose0"]], res, jac))
    # 3. preintegration 0 -> 1
    imu = make_imu_segment(rng, 100)
    st = random_state(rng)
    st["p"], st["q"] = poses[0, :3], poses[0, 3:]
    st["v"], st["bg"], st["ba"] = mixes[0, :3], mixes[0, 3:6], mixes[0, 6:]
    res, jac = ev.preint(imu, st, poses[0], mixes[0], poses[1], mixes[1])
    facs.append(([bid["pose0"], bid["mix0"], bid["pose1"], bid["mix1"]], res, jac))
    # 4. reprojection factors of the landmarks referenced in keyframe 0
    res, jac = ev.reproj(ba["consts"], ba["params"], ba["offs"])
    for f, o in enumerate(ba["offs"]):
        k = int(o[1]) // 7
        j = int(o[3]) - (7 * n_kf + 7)
        facs.append(([bid["pose0"], bid[f"pose{k}"], bid["ext"], bid[f"invdepth{j}"], bid["td"]], res[f], jac[f]))
    # local indices: marginalized first
    used = sorted({b for f in facs for b in f[0]})
    marg = [bid["pose0"], bid["mix0"]] + [bid[f"invdepth{j}"] for j in range(n_lm)]
    rem = [b for b in used if b not in set(marg)]
    index = np.full(len(names), -1, np.int32)
    o = 0
    for b in marg + rem:
        index[b] = o
        o += 6 if size[b] == 7 else size[b]
    m = sum(6 if size[b] == 7 else size[b] for b in marg)
    # compact block table to the used blocks
    remap = {b: i for i, b in enumerate(used)}
    nres, blk_off, blk, res_off, jac_off, data = [], [0], [], [], [], []
    pos = 0
    for bl, r_, j_ in facs:
        r_, j_ = np.asarray(r_, np.float64).ravel(), np.asarray(j_, np.float64).ravel()
        nres.append(r_.size)
        blk += [remap[b] for b in bl]
        blk_off.append(len(blk))
        res_off.append(pos)
        jac_off.append(pos + r_.size)
        data += [r_, j_]
        pos += r_.size + j_.size
    loss = None
    if huber is not None:
        loss = np.array([huber if len(bl) == 5 else 0.0 for bl, _, _ in facs])
    return dict(nres=np.array(nres, np.int32), blk_off=np.array(blk_off, np.int32), blk=np.array(blk, np.int32),
                res_off=np.array(res_off, np.int64), jac_off=np.array(jac_off, np.int64),
                data=np.concatenate(data), loss=loss, size=np.array([size[b] for b in used], np.int32),
                index=index[used], m=int(m), L=int(o), names=[names[b] for b in used])


class DeviceFactorEvaluator:
    """make_marg_problem's evaluator on the device (gvx.Context factor entry points)."""

    def __init__(self, ctx):
        self.ctx = ctx

    def reproj(self, consts, params, offs):
        from gvx import REPROJ_DTYPE
        return self.ctx.reproj_eval(np.asarray(consts).astype(REPROJ_DTYPE), params, offs)

    def preint(self, imu, st, p0, m0, p1, m1):
        from gvx import STATE_DTYPE as GS
        gs = np.zeros(1, GS)
        for k in ("time", "p", "q", "v", "bg", "ba"):
            gs[k] = st[k]
        iewn = np.zeros((1, 3))
        out, pn, pn_off = self.ctx.preint_integrate(2, imu_params(), [imu], gs, iewn)
        params = np.concatenate([p0, m0, p1, m1])
        res, jac = self.ctx.preint_factor_eval(out, pn, pn_off, params, np.array([[0, 7, 16, 23]], np.int32))
        return res[0], jac[0]

    def gnss(self, consts, pose):
        res, jac = self.ctx.small_factor_eval(0, consts.reshape(1, -1), pose, np.array([0], np.int32))
        return res[0], jac[0]

    def marg(self, size, index, xoff, x0, x, J0, e0):
        return self.ctx.marg_factor_eval(size, index, xoff, x0, x, J0, e0)


def lm_problem(p):
    """A make_marg_problem problem re-laid-out for the LM step (gvx_schur_solve,
    Ceres' DENSE_SCHUR): the e-blocks (inverse depths) at local indices [0, m), the
    other blocks after them in block order."""
    names = p["names"]
    size = p["size"]
    e = [b for b, n in enumerate(names) if n.startswith("invdepth")]
    f = [b for b, n in enumerate(names) if not n.startswith("invdepth")]
    index = np.zeros(len(names), np.int32)
    o = 0
    for b in e + f:
        index[b] = o
        o += 6 if size[b] == 7 else size[b]
    m = sum(int(size[b]) for b in e)
    return dict(p, index=index, m=int(m), L=int(o))


def dense_normal_equations(p):
    """(J^T J, -J^T r) of a problem dict in its local indices, from the dense
    stacked Jacobian (pose blocks: the first 6 of their 7 columns) -- the numpy
    check of gvx_schur_solve / marginalize's constructEquation."""
    L = int(p["L"])
    rows = int(np.sum(p["nres"]))
    J = np.zeros((rows, L))
    r = np.zeros(rows)
    row = 0
    data = p["data"]
    for f in range(len(p["nres"])):
        R = int(p["nres"][f])
        r[row:row + R] = data[p["res_off"][f]:p["res_off"][f] + R]
        off = int(p["jac_off"][f])
        for b in p["blk"][p["blk_off"][f]:p["blk_off"][f + 1]]:
            s = int(p["size"][b])
            Jb = data[off:off + R * s].reshape(R, s)
            loc = 6 if s == 7 else s
            J[row:row + R, p["index"][b]:p["index"][b] + loc] = Jb[:, :loc]
            off += R * s
        row += R
    return J.T @ J, -J.T @ r
