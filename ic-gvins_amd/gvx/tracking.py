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


class DeviceSequenceTracker:
    """SequenceTracker's loop with the tracker state on the device
    (gvx_track_frame_dev): no host round trip per frame.

    frames (optional): the whole sequence resident in HBM ([F, h, w] u8 tensor).
    The frame to process is then picked on the device (gvx_frame_preprocess_indexed_dev
    at a device-held frame index) and every frame's track list is appended to
    self.rec_tracks / self.rec_counts (gvx_track_record_dev, which advances the
    index), so with graph=True a frame is exactly one graph launch: the work
    (CLAHE + pyramid + LK + FB + compaction + detection top-up + record) is
    captured once per frame parity (the two cached frame ids
    alternate) and replayed.  Without frames, step(d_frame) takes the frame's
    device pointer (copied into a fixed staging buffer first in graph mode)."""

    def __init__(self, ctx: Context, w: int, h: int, n_features: int = 150,
                 klt: Optional[KltParams] = None, detect: Optional[DetectParams] = None,
                 ids=(0, 1), graph: bool = False, device=None, frames=None, pipeline: bool = False,
                 eig_branch: bool = False, batch: int = 1):
        import torch
        self.ctx, self.w, self.h, self.n = ctx, w, h, n_features
        self.kp = klt or KltParams.default()
        self.dp = detect or DetectParams.default(max_features=n_features)
        self.ids = ids
        self.t = 0
        dev = device or torch.device("cuda")
        f32 = dict(dtype=torch.float32, device=dev)
        self.pts = torch.zeros((n_features, 2), **f32)
        self.vel = torch.zeros((n_features, 2), **f32)
        self.init = torch.zeros((n_features, 2), **f32)
        self.count = torch.zeros(1, dtype=torch.int32, device=dev)
        self.graph = graph
        self.graphs = {}
        self.frames = frames
        self.stage = torch.empty((h, w), dtype=torch.uint8, device=dev) if (graph and frames is None) else None
        # pipeline (HBM-resident sequences only): frame t+1's preprocessing
        # (CLAHE + pyramid into a third frame slot) runs as a side branch beside
        # frame t's tracking (gvx_branch_begin / _end / _join), reading the frame
        # at its own device counter.  At t = F - 1 that counter is past the last
        # frame: the device clamps it (the spare preprocessing is never tracked).
        self.pipeline = bool(pipeline) and frames is not None
        # eig_branch (pipelined only): the detection's eigenvalue map of every block
        # on the preprocessing branch (gvx_frame_eig_dev) instead of the tiles of the
        # detecting blocks in the tracking graph
        self.eig_branch = bool(eig_branch) and self.pipeline
        # batch (pipelined only): frames go to the device K = batch at a time -- a
        # graph preprocessing K frames on the side branch beside a graph tracking the
        # previous K (3 sets of K frame slots rotating), so the branch fork / join
        # and the graph launches are paid once per K frames instead of per frame
        # (tools/graph_probe.hip: a stream-pair fork/join costs ~13-15 us per frame)
        self.batch = max(1, int(batch)) if self.pipeline else 1
        if self.pipeline:
            need = 3 * self.batch
            base = max(self.ids) + 1
            self.ids = tuple(self.ids)[:need] + tuple(range(base, base + max(0, need - len(self.ids))))
            self.pindex = torch.full((1,), 0 if self.batch > 1 else 1, dtype=torch.int32, device=dev)
        if frames is not None:
            F = frames.shape[0]
            self.index = torch.zeros(1, dtype=torch.int32, device=dev)
            self.rec_tracks = torch.zeros((F, n_features, 2), **f32)
            self.rec_counts = torch.zeros(F, dtype=torch.int32, device=dev)

    def _pre_next(self, t: int):
        # frame *pindex (= t + 1) into the slot of frame t+1; the branch advances its
        # own counter, so it never reads the index the tracking graph's record advances
        self.ctx.frame_preprocess_indexed_dev(self.ids[(t + 1) % 3], self.frames.data_ptr(), self.w * self.h,
                                              self.pindex.data_ptr(), self.frames.shape[0], self.w, self.h,
                                              params=self.kp)
        # the detection's eigenvalue map of frame t+1 on this branch too: it depends
        # on the image alone, so frame t+1's tracking only selects
        if self.eig_branch:
            self.ctx.frame_eig_dev(self.ids[(t + 1) % 3], detect=self.dp)
        self.ctx.index_advance_dev(self.pindex.data_ptr(), 1)

    def _track_cur(self, t: int):
        self.ctx.track_frame_record_dev(self.ids[(t - 1) % 3], self.ids[t % 3], t > 0, self.pts.data_ptr(),
                                        self.vel.data_ptr(), self.init.data_ptr(), self.count.data_ptr(), self.n,
                                        self.w, self.h, self.rec_tracks.data_ptr(), self.rec_counts.data_ptr(),
                                        self.index.data_ptr(), self.frames.shape[0], klt=self.kp, detect=self.dp)

    def _graph(self, key, fn, t: int):
        g = self.graphs.get(key)
        if g is None:
            g = self.graphs[key] = self.ctx.capture(fn, t)
        return g

    def _enqueue_pipelined(self, t: int, graphs: bool):
        """Frame t+1's preprocessing on the context's side branch beside frame t's
        tracking (+ its record).  Frame t's tracking waits for frame t's
        preprocessing (the join at the top); frame t+1's preprocessing waits for
        frame t-1's tracking, the last reader of the slot it writes (the fork).
        With graphs, each half is its own captured graph (one per frame-slot
        rotation), launched on its own stream: the branches of ONE captured graph
        measured serialised (r02 v21)."""
        ctx = self.ctx
        if t == 0:
            ctx.frame_preprocess_indexed_dev(self.ids[0], self.frames.data_ptr(), self.w * self.h,
                                             self.index.data_ptr(), self.frames.shape[0], self.w, self.h,
                                             params=self.kp)
            if self.eig_branch:
                ctx.frame_eig_dev(self.ids[0], detect=self.dp)
        ctx.branch_join()
        if graphs:
            ga = self._graph(("pre", t % 3), self._pre_next, t)
            gb = self._graph(("trk", t % 3), self._track_cur, t)
        ctx.branch_begin()
        ctx.graph_launch(ga) if graphs else self._pre_next(t)
        ctx.branch_end()
        ctx.graph_launch(gb) if graphs else self._track_cur(t)

    def _set(self, b: int):
        K = self.batch
        return self.ids[(b % 3) * K:(b % 3 + 1) * K]

    def _batch_len(self, b: int) -> int:
        return min(self.batch, self.frames.shape[0] - b * self.batch)

    def _pre_batch(self, b: int):
        # frames b*K .. b*K + len - 1 (read at the branch's own counter) into set b % 3
        for fid in self._set(b)[:self._batch_len(b)]:
            self.ctx.frame_preprocess_indexed_dev(fid, self.frames.data_ptr(), self.w * self.h,
                                                  self.pindex.data_ptr(), self.frames.shape[0], self.w, self.h,
                                                  params=self.kp)
            if self.eig_branch:
                self.ctx.frame_eig_dev(fid, detect=self.dp)
            self.ctx.index_advance_dev(self.pindex.data_ptr(), 1)

    def _trk_batch(self, b: int):
        cur, prv = self._set(b), self._set(b - 1)
        for i in range(self._batch_len(b)):
            t = b * self.batch + i
            self.ctx.track_frame_record_dev(cur[i - 1] if i else prv[-1], cur[i], t > 0, self.pts.data_ptr(),
                                            self.vel.data_ptr(), self.init.data_ptr(), self.count.data_ptr(), self.n,
                                            self.w, self.h, self.rec_tracks.data_ptr(), self.rec_counts.data_ptr(),
                                            self.index.data_ptr(), self.frames.shape[0], klt=self.kp, detect=self.dp)

    def _enqueue_batch(self, b: int):
        """Batch b: join the branch that preprocessed it, fork the preprocessing of
        batch b+1 (after batch b-1's tracking, the last reader of its slots), then
        batch b's tracking.  Whole batches replay captured graphs once every set's
        slots exist (batch >= 3); a short last batch runs eagerly."""
        ctx, K = self.ctx, self.batch
        nb = (self.frames.shape[0] + K - 1) // K
        if b == 0:
            self._pre_batch(0)
        ctx.branch_join()
        # graphs are captured with no branch open
        gp = gt = None
        if self.graph and b + 1 < nb and b + 1 >= 3 and self._batch_len(b + 1) == K:
            gp = self._graph(("preK", (b + 1) % 3), self._pre_batch, b + 1)
        if self.graph and b >= 3 and self._batch_len(b) == K:
            gt = self._graph(("trkK", b % 3), self._trk_batch, b)
        if b + 1 < nb:
            ctx.branch_begin()
            ctx.graph_launch(gp) if gp is not None else self._pre_batch(b + 1)
            ctx.branch_end()
        ctx.graph_launch(gt) if gt is not None else self._trk_batch(b)

    def _enqueue(self, d_frame: Optional[int], t: int):
        if self.pipeline:
            return self._enqueue_pipelined(t, False)
        ctx = self.ctx
        cur, prev = self.ids[t % 2], self.ids[(t - 1) % 2]
        if self.frames is not None:
            # frame *index of the HBM-resident sequence, equalised straight into the
            # frame cache (no staging copy)
            ctx.frame_preprocess_indexed_dev(cur, self.frames.data_ptr(), self.w * self.h, self.index.data_ptr(),
                                             self.frames.shape[0], self.w, self.h, params=self.kp)
        else:
            ctx.frame_preprocess_dev(cur, d_frame, self.w, self.h, None, params=self.kp)
        if self.frames is not None:
            # the frame and its track-list record (appended by the detection's
            # last kernel, which advances the frame index)
            ctx.track_frame_record_dev(prev, cur, t > 0, self.pts.data_ptr(), self.vel.data_ptr(),
                                       self.init.data_ptr(), self.count.data_ptr(), self.n, self.w, self.h,
                                       self.rec_tracks.data_ptr(), self.rec_counts.data_ptr(), self.index.data_ptr(),
                                       self.frames.shape[0], klt=self.kp, detect=self.dp)
        else:
            ctx.track_frame_dev(prev, cur, t > 0, self.pts.data_ptr(), self.vel.data_ptr(), self.init.data_ptr(),
                                self.count.data_ptr(), self.n, self.w, self.h, klt=self.kp, detect=self.dp)

    def step(self, d_frame: Optional[int] = None) -> None:
        """Enqueue one frame (nothing waits); the tracks are
        self.pts[:self.count] once the stream has run it."""
        t = self.t
        if self.frames is not None and t >= self.frames.shape[0]:
            raise IndexError(f"step {t}: the resident sequence has {self.frames.shape[0]} frames")
        if self.frames is None and d_frame is None:
            raise ValueError("step() needs the frame's device pointer when no sequence is resident")
        if self.batch > 1:
            # frames t .. t + K - 1 are enqueued together at the first of them
            if t % self.batch == 0:
                self._enqueue_batch(t // self.batch)
        elif not self.graph or t < 3:
            self._enqueue(d_frame, t)  # the first frames also size every buffer
        elif self.pipeline:
            self._enqueue_pipelined(t, True)
        else:
            if self.frames is None:
                self.ctx.copy_dev(self.stage.data_ptr(), d_frame, self.w * self.h)
            key = t % 2  # the frame slots' rotation
            g = self.graphs.get(key)
            if g is None:
                src = None if self.frames is not None else self.stage.data_ptr()
                g = self.graphs[key] = self.ctx.capture(lambda tt: self._enqueue(src, tt), t)
            self.ctx.graph_launch(g)
        self.t += 1

    def tracks(self) -> np.ndarray:
        """The current track list (synchronises)."""
        self.ctx.sync()
        n = int(self.count.cpu()[0])
        return self.pts[:n].cpu().numpy()

    def close(self):
        if self.pipeline:
            self.ctx.branch_join()  # the last frame's preprocessing branch
        for g in self.graphs.values():
            g.destroy()
        self.graphs = {}
