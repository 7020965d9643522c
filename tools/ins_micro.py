"""INS mechanization throughput (csrc/ins.hip): n chains x m IMU samples through
gvx_ins_propagate_dev with inputs resident in HBM, device time from the
context's profiling events; plus one redoInsMechanization window through the
host entry (its latency, PCIe round trip included).  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ic-gvins_amd"))


def main(n=4096, m=400, reps=20):
    import torch
    import gvx
    from gvx import synth_ba
    torch.cuda.init()
    ctx = gvx.Context(0)
    rng = np.random.default_rng(1)
    seg = synth_ba.make_imu_segment(rng, m)
    imu = np.tile(seg, n)
    off = (np.arange(n + 1) * m).astype(np.int32)
    st0 = np.array([synth_ba.random_state(rng, float(seg[0]["time"]))] * n)
    dev = torch.device("cuda", 0)
    d_imu = torch.from_numpy(imu.view(np.uint8).copy()).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_s0 = torch.from_numpy(st0.view(np.uint8).copy()).to(dev)
    d_st = torch.empty(n * m * gvx.STATE_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    cfg = gvx.InsConfig.make(True, (0, 0, 9.7803267715), gvx.earth_iewn(np.zeros(3), (0.5, 0.2, 10.0)))
    torch.cuda.synchronize()

    def run():
        ctx.ins_propagate_dev(cfg, n, d_imu.data_ptr(), d_off.data_ptr(), d_s0.data_ptr(), d_st.data_ptr())

    for _ in range(3):
        run()
    ctx.sync()
    ctx.profile_reset()
    ctx.profile(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    ctx.sync()
    el = time.perf_counter() - t0
    ms, _ = ctx.profile_read("ins")
    ctx.profile(False)
    steps = n * (m - 1) * reps
    io = n * m * (gvx.IMU_DTYPE.itemsize + gvx.STATE_DTYPE.itemsize)  # bytes per launch
    # one redo window (the reference's per-optimisation call): 200 samples
    win = seg[:200]
    states = np.zeros(200, gvx.STATE_DTYPE)
    upd = st0[0].copy()
    upd["time"] = float(win[40]["time"]) + 0.0021
    ctx.redo_ins_mechanization(cfg, upd, win, states)
    t1 = time.perf_counter()
    for _ in range(50):
        ctx.redo_ins_mechanization(cfg, upd, win, states)
    redo_us = (time.perf_counter() - t1) / 50 * 1e6
    print(json.dumps({"chains": n, "samples_per_chain": m, "steps_per_s": round(steps / el),
                      "device_ms_per_launch": round(ms / reps, 4),
                      "device_steps_per_s": round(steps / (ms * 1e-3)),
                      "io_gb_s": round(io * reps / (ms * 1e-3) / 1e9, 1),
                      "redo_window_200_us": round(redo_us, 1)}))
    ctx.close()


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
