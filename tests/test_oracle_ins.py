"""The CPU restatement of the INS mechanization and IMU-series extraction
(oracle/ins.c; misc.cc:40-384 of the reference) against closed forms and
self-consistency.  Eigen is absent, so it is "parity unpinned" against the
reference binaries."""
import numpy as np
import pytest

import oracle as orc

G = 9.7803267715
DT = 0.005


def _imu(n, dtheta=(0, 0, 0), dvel=(0, 0, 0), t0=10.0):
    imu = np.zeros(n, orc.IMU_DTYPE)
    imu["time"] = t0 + DT * np.arange(n)
    imu["dt"] = DT
    imu["dtheta"] = np.asarray(dtheta, float) * DT
    imu["dvel"] = np.asarray(dvel, float) * DT
    return imu


def _cfg(earth=False, iewn=(0, 0, 0)):
    return orc.InsConfig.make(earth, (0, 0, G), iewn)


def test_stationary_stays_put():
    # specific force of a level, stationary IMU: -g along z (NED, g positive down)
    imu = _imu(200, dvel=(0, 0, -G))
    st = orc.ins_propagate(_cfg(), imu, orc.make_state(imu[0]["time"]))
    assert np.abs(st["p"]).max() < 1e-12 and np.abs(st["v"]).max() < 1e-12
    assert np.allclose(st["q"][-1], [0, 0, 0, 1], atol=1e-15)
    assert np.array_equal(st["time"], imu["time"])


def test_constant_acceleration_closed_form():
    a = np.array([0.3, -0.2, 0.1])
    imu = _imu(101, dvel=a - np.array([0, 0, G]))
    st = orc.ins_propagate(_cfg(), imu, orc.make_state(imu[0]["time"]))
    t = 100 * DT
    assert np.allclose(st["v"][-1], a * t, rtol=1e-12, atol=1e-14)
    assert np.allclose(st["p"][-1], 0.5 * a * t * t, rtol=1e-10, atol=1e-14)


def test_constant_rate_rotation():
    w = 0.4  # rad/s about z, no coning for a fixed axis
    imu = _imu(201, dtheta=(0, 0, w), dvel=(0, 0, -G))
    st = orc.ins_propagate(_cfg(), imu, orc.make_state(imu[0]["time"]))
    ang = w * 200 * DT
    assert np.allclose(st["q"][-1], [0, 0, np.sin(ang / 2), np.cos(ang / 2)], atol=1e-13)


def test_earth_with_zero_rate_equals_normal():
    from gvx import synth_ba
    imu = synth_ba.make_imu_segment(np.random.default_rng(3), 80)
    s0 = orc.make_state(float(imu[0]["time"]), (1, 2, 3), (0.1, -0.2, 0.05, 0.97), (5, 0.1, 0), (1e-4, 0, -2e-4),
                        (0.01, -0.02, 0.0))
    a = orc.ins_propagate(_cfg(False), imu, s0)
    b = orc.ins_propagate(_cfg(True, (0, 0, 0)), imu, s0)
    for k in ("p", "q", "v"):
        assert np.allclose(a[k], b[k], rtol=0, atol=1e-12)


def _window(n=120, seed=5):
    from gvx import synth_ba
    imu = synth_ba.make_imu_segment(np.random.default_rng(seed), n)
    s = orc.make_state(float(imu[0]["time"]), (0, 0, 0), (0, 0, 0, 1), (3, 0, 0), (1e-4, 0, 0), (0, 0.01, 0))
    return imu, s


@pytest.mark.parametrize("offset,need", [(0.0021, 2), (0.00003, -1), (0.00499, 1)])
def test_redo_matches_manual_chain(offset, need):
    imu, s = _window()
    cfg = _cfg(True, orc.earth_iewn(np.zeros(3), (0.5, 0.2, 10.0)))
    states = np.zeros(len(imu), orc.STATE_DTYPE)
    t = float(imu[40]["time"]) + offset
    s.time = t
    assert orc.ins_window_index(imu, len(imu), t) == 41
    assert orc.lib().orc_need_interpolation(imu[40:41].ctypes.data, imu[41:42].ctypes.data, t) == need
    idx = orc.redo_ins_mechanization(cfg, s, imu, states)
    assert idx == 41
    # the same chain by hand: a series starting with the split sample, then the window
    if need == 2:
        part = imu[41:].copy()
        head = imu[41:42].copy()
        scale = (head["time"][0] - t) / head["dt"][0]
        first = head.copy()
        first["time"], first["dt"] = t, head["dt"][0] - (head["time"][0] - t)
        first["dtheta"], first["dvel"] = head["dtheta"] * (1 - scale), head["dvel"] * (1 - scale)
        part[0]["dt"] = head["time"][0] - t
        part[0]["dtheta"], part[0]["dvel"] = head["dtheta"][0] * scale, head["dvel"][0] * scale
        series = np.concatenate([first, part])
        ref = orc.ins_propagate(cfg, series, s)[1:]
    elif need == -1:
        ref = orc.ins_propagate(cfg, imu[40:], s)[1:]
    else:
        s1 = orc.make_state(float(imu[41]["time"]), s.p, s.q, s.v, s.bg, s.ba)
        ref = orc.ins_propagate(cfg, imu[41:], s1)
    for k in ("time", "p", "q", "v"):
        assert np.array_equal(states[41:][k], ref[k]), k
    assert np.all(states[:41]["time"] == 0)  # untouched


def test_redo_out_of_window():
    imu, s = _window()
    s.time = float(imu[-1]["time"]) + 1.0
    states = np.zeros(len(imu), orc.STATE_DTYPE)
    assert orc.redo_ins_mechanization(_cfg(), s, imu, states) == 0 and not states["time"].any()


def test_imu_series_from_to():
    imu, _ = _window()
    t0, t1 = float(imu[10]["time"]) + 0.002, float(imu[60]["time"]) + 0.0031
    ser = orc.imu_series_from_to(imu, t0, t1)
    assert ser[0]["time"] == t0 and ser[-1]["time"] == t1
    # the split samples keep the increments: the series integrates exactly the window over [t0, t1]
    full = imu[11:61]["dtheta"].sum(0)
    tail = imu[61]["dtheta"] * (1 - (imu[61]["time"] - t1) / imu[61]["dt"])
    assert np.allclose(ser["dtheta"].sum(0), full + tail, rtol=1e-12, atol=1e-18)
    assert len(ser) == 1 + 50 + 1
    assert orc.imu_series_from_to(imu, t0, float(imu[-1]["time"]) + 1) is None
