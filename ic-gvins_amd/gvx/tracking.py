"""Per-frame image path of IC-GVINS's Tracking::track on the device.

The reference processes every new frame as (tracking/tracking.cc):
  * preprocessing: CLAHE (createCLAHE(3.0, 21x21)->apply, :63, :139);
  * track the previous frame's points into the new frame: forward and backward
    calcOpticalFlowPyrLK with OPTFLOW_USE_INITIAL_FLOW, then the FB / border /
    status filter and reduceVector (:380-408, :831-849);
  * top the tracks up with block-grid detection (featuresDetection, :576-688)
    when fewer than track_max_features_ remain (:220, :259).
SequenceTracker runs exactly that order on libgvx (one cached pyramid per frame,
built once and reused by both LK directions).  The initial flow is the
constant-velocity prediction of the last motion (the reference predicts with
the IMU rotation; the synthetic sequences have no IMU).  Everything here is the
product path: it calls libgvx only and raises GvxError when it is missing.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from . import Context, DetectParams, KltParams


class SequenceTracker:
    """One sequence on one context.  Frames alternate between two cached frame
    ids, so the previous frame's pyramid stays resident while the new one is
    built."""

    def __init__(self, ctx: Context, w: int, h: int, n_features: int = 150,
                 klt: Optional[KltParams] = None, detect: Optional[DetectParams] = None,
                 ids=(0, 1)):
        self.ctx, self.w, self.h, self.n = ctx, w, h, n_features
        self.kp = klt or KltParams.default()
        self.dp = detect or DetectParams.default(max_features=n_features)
        self.ids = ids
        self.t = 0
        self.pts = np.zeros((0, 2), np.float32)
        self.vel = np.zeros((0, 2), np.float32)
        self.last = {}  # per-frame record of the last step (tracking + detection outputs)

    def step(self, d_frame: int, stride: Optional[int] = None) -> np.ndarray:
        """Process one frame (device pointer to h x w u8) -> the frame's tracks
        [n, 2] f32 (kept tracks first, in their order, then new corners)."""
        ctx, t = self.ctx, self.t
        cur, prev = self.ids[t % 2], self.ids[(t - 1) % 2]
        rec = {}
        # Tracking::preprocessing (CLAHE) + the frame's pyramid, once
        ctx.frame_preprocess_dev(cur, d_frame, self.w, self.h, stride, params=self.kp)
        pts, vel = self.pts, self.vel
        if t > 0 and pts.shape[0]:
            r = ctx.track_fb(prev, cur, pts, pts + vel, self.w, self.h, params=self.kp)
            k = r["kept_idx"]
            nxt = r["next"][k]
            vel = nxt - pts[k]
            pts = nxt
            rec["track"] = r
        if pts.shape[0] < self.n:
            corners, _ = ctx.detect(cur, pts, pts, True, int(pts.shape[0]), self.dp)
            rec["corners"] = corners
            if corners is not None and corners.shape[0]:
                add = corners[:self.n - pts.shape[0]]
                pts = np.concatenate([pts, add]).astype(np.float32)
                vel = np.concatenate([vel, np.zeros_like(add)]).astype(np.float32)
        self.pts, self.vel = pts, vel
        self.last = rec
        self.t += 1
        return pts
