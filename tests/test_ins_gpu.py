"""INS mechanization on the device (csrc/ins.hip through gvx_ins_propagate /
gvx_redo_ins_mechanization) against the CPU restatement (oracle/ins.c;
MISC::insMechanization / redoInsMechanization, misc.cc:174-284).

Tolerance: fp64, 1e-10 relative (+1e-12 absolute) per state component -- device
and host differ only in sin/cos (ocml vs glibc) inside rotvec2quaternion; times
and biases are copied, so they must match exactly."""
import numpy as np
import pytest

from gvx import synth_ba

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-10, 1e-12
G = 9.7803267715


def _ostate(s):
    import oracle as orc
    return orc.make_state(float(s["time"]), s["p"], s["q"], s["v"], s["bg"], s["ba"])


def _cfgs(gvx_mod, orc, earth):
    iewn = orc.earth_iewn(np.zeros(3), (0.5, 0.2, 10.0)) if earth else np.zeros(3)
    return gvx_mod.InsConfig.make(earth, (0, 0, G), iewn), orc.InsConfig.make(earth, (0, 0, G), iewn)


def _close(a, b, what):
    assert np.array_equal(a["time"], b["time"]), what + ": time"
    for k in ("p", "q", "v"):
        np.testing.assert_allclose(a[k], b[k], rtol=RTOL, atol=ATOL, err_msg=f"{what}: {k}")
    for k in ("bg", "ba"):
        assert np.array_equal(a[k], b[k]), f"{what}: {k}"


@pytest.mark.parametrize("earth", [False, True])
def test_propagate_chains_match_oracle(ctx, gvx_mod, orc, earth):
    rng = np.random.default_rng(41 + earth)
    lens = (1, 2, 3, 64, 65, 66, 129, 150, 400)  # around the 64-step LDS chunks
    segs = [synth_ba.make_imu_segment(rng, m, t0=float(i)) for i, m in enumerate(lens)]
    st0 = np.array([synth_ba.random_state(rng, float(s[0]["time"])) for s in segs])
    gcfg, ocfg = _cfgs(gvx_mod, orc, earth)
    out = ctx.ins_propagate(gcfg, segs, st0)
    assert len(out) == len(segs)
    for i, (seg, got) in enumerate(zip(segs, out)):
        ref = orc.ins_propagate(ocfg, seg, _ostate(st0[i]))
        _close(got, ref, f"chain {i} (m={len(seg)})")


def test_propagate_empty_and_zero_length(ctx, gvx_mod, orc):
    gcfg, _ = _cfgs(gvx_mod, orc, False)
    assert ctx.ins_propagate(gcfg, [], np.zeros(0, gvx_mod.STATE_DTYPE)) == []
    rng = np.random.default_rng(3)
    seg = synth_ba.make_imu_segment(rng, 10)
    s = synth_ba.random_state(rng, float(seg[0]["time"]))
    out = ctx.ins_propagate(gcfg, [seg[:0], seg], np.array([s, s]))
    assert len(out[0]) == 0 and len(out[1]) == 10


def test_stationary_closed_form_on_device(ctx, gvx_mod, orc):
    imu = np.zeros(300, gvx_mod.IMU_DTYPE)
    imu["time"] = 5.0 + 0.005 * np.arange(300)
    imu["dt"] = 0.005
    imu["dvel"][:, 2] = -G * 0.005
    gcfg, _ = _cfgs(gvx_mod, orc, False)
    s0 = np.zeros((), gvx_mod.STATE_DTYPE)
    s0["time"], s0["q"] = 5.0, (0, 0, 0, 1)
    st = ctx.ins_propagate(gcfg, [imu], np.array([s0]))[0]
    assert np.abs(st["p"]).max() < 1e-12 and np.abs(st["v"]).max() < 1e-12
    assert np.array_equal(st["time"], imu["time"])


@pytest.mark.parametrize("earth", [False, True])
@pytest.mark.parametrize("offset,need", [(0.0021, 2), (0.00003, -1), (0.00499, 1), (0.0, 0)])
def test_redo_matches_oracle(ctx, gvx_mod, orc, earth, offset, need):
    rng = np.random.default_rng(7)
    imu = synth_ba.make_imu_segment(rng, 200, t0=100.0)
    gcfg, ocfg = _cfgs(gvx_mod, orc, earth)
    upd = synth_ba.random_state(rng)
    t = float(imu[40]["time"]) + offset
    upd["time"] = t
    idx = orc.ins_window_index(imu, len(imu), t)
    assert orc.lib().orc_need_interpolation(imu[idx - 1:idx].ctypes.data, imu[idx:idx + 1].ctypes.data, t) == need
    base = np.array([synth_ba.random_state(rng, float(x)) for x in imu["time"]])
    ref, got = base.copy(), base.copy()
    iref = orc.redo_ins_mechanization(ocfg, _ostate(upd), imu, ref)
    igot = ctx.redo_ins_mechanization(gcfg, upd, imu, got)
    assert igot == iref == idx
    assert np.array_equal(got[:idx], base[:idx])  # untouched before the index
    _close(got, ref, f"redo need={need}")


def test_redo_out_of_window(ctx, gvx_mod, orc):
    rng = np.random.default_rng(9)
    imu = synth_ba.make_imu_segment(rng, 50, t0=3.0)
    gcfg, _ = _cfgs(gvx_mod, orc, False)
    upd = synth_ba.random_state(rng, float(imu[-1]["time"]) + 1.0)
    st = np.zeros(len(imu), gvx_mod.STATE_DTYPE)
    assert ctx.redo_ins_mechanization(gcfg, upd, imu, st) == 0
    assert not st["time"].any()


def test_propagate_dev_matches_host_entry(ctx, gvx_mod, orc):
    import torch
    rng = np.random.default_rng(12)
    segs = [synth_ba.make_imu_segment(rng, m, t0=float(i)) for i, m in enumerate((90, 33, 200))]
    st0 = np.array([synth_ba.random_state(rng, float(s[0]["time"])) for s in segs])
    gcfg, _ = _cfgs(gvx_mod, orc, True)
    host = ctx.ins_propagate(gcfg, segs, st0)
    imu = np.concatenate(segs)
    off = np.zeros(len(segs) + 1, np.int32)
    off[1:] = np.cumsum([len(s) for s in segs])
    dev = torch.device("cuda", 0)
    d_imu = torch.from_numpy(imu.view(np.uint8).copy()).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_s0 = torch.from_numpy(st0.view(np.uint8).copy()).to(dev)
    d_st = torch.empty(len(imu) * gvx_mod.STATE_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    ctx.ins_propagate_dev(gcfg, len(segs), d_imu.data_ptr(), d_off.data_ptr(), d_s0.data_ptr(), d_st.data_ptr())
    ctx.sync()
    got = d_st.cpu().numpy().view(gvx_mod.STATE_DTYPE)
    assert np.array_equal(got, np.concatenate(host))
