"""configs[4]: the sequence replay's per-frame loop on the GPU
against the same loop on the oracle, frame by frame.

Tracking::track's image path (tracking/tracking.cc:107-245): CLAHE (:139) ->
pyramid -> forward + backward LK with the initial flow (:385, :390) -> FB /
border / status filter + reduceVector (:396-408, :831-849) -> block-grid
detection topping the tracks up to track_max_features_ (:220, :576-688).
gvx.tracking.SequenceTracker runs it on libgvx; `_oracle_sequence` below runs the
same order on the C restatement.  Per frame the forward/backward flow, status,
keep flags and kept indices must be bit-exact, and so must the detected corners
and the resulting track list (the frames are rendered once on the device and
copied to the host for the oracle)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, N, L = 1280, 560, 150, 3


def _oracle_sequence(orc, frames, kp, dp, nthreads=1, equalised=None):
    """The oracle's Tracking::track loop; `equalised` (optional): the frames'
    CLAHE outputs computed beforehand (they depend on the frame alone)."""
    pts, vel = np.zeros((0, 2), np.float32), np.zeros((0, 2), np.float32)
    prev_eq = None
    out = []
    for t, f in enumerate(frames):
        eq = orc.clahe(f) if equalised is None else equalised[t]
        rec = {}
        if t > 0 and pts.shape[0]:
            # each pyramid built once (bit-identical to OpenCV's per-call rebuild)
            r = orc.klt_fb(prev_eq, eq, pts, pts + vel, params=kp, reuse_pyramids=nthreads > 1, nthreads=nthreads)
            k = r["kept_idx"]
            nxt = r["next"][k]
            vel = nxt - pts[k]
            pts = nxt
            rec["track"] = r
        if pts.shape[0] < N:
            corners, _ = orc.features_detection(eq, pts, pts, True, int(pts.shape[0]), dp)
            rec["corners"] = corners
            if corners is not None and corners.shape[0]:
                add = corners[:N - pts.shape[0]]
                pts = np.concatenate([pts, add]).astype(np.float32)
                vel = np.concatenate([vel, np.zeros_like(add)]).astype(np.float32)
        rec["pts"] = pts.copy()
        out.append(rec)
        prev_eq = eq
    return out


@pytest.mark.parametrize("n_frames", [30])
def test_sequence_replay_bit_exact(ctx, orc, gvx_mod, n_frames):
    import torch
    from gvx import synth
    from gvx.tracking import SequenceTracker
    dev = torch.device("cuda", 0)
    frames, _ = synth.make_sequence(W, H, n_frames, dev, seed=synth.SEED)
    host = frames.cpu().numpy()
    kp = gvx_mod.KltParams.default(max_level=L)
    dp = gvx_mod.DetectParams.default(max_features=N)
    okp = orc.KltParams.default(max_level=L)
    odp = orc.DetectParams.default() if hasattr(orc.DetectParams, "default") else None
    ref = _oracle_sequence(orc, host, okp, odp)
    tr = SequenceTracker(ctx, W, H, N, klt=kp, detect=dp)
    n_tracked = n_detect = 0
    for t in range(n_frames):
        pts = tr.step(frames[t].data_ptr())
        g, o = tr.last, ref[t]
        assert ("track" in g) == ("track" in o), f"frame {t}: tracking ran on one side only"
        if "track" in g:
            for k in ("next", "back", "st_f", "st_b", "keep", "kept_idx"):
                assert np.array_equal(g["track"][k], o["track"][k]), f"frame {t}: {k}"
            n_tracked += len(g["track"]["kept_idx"])
        assert ("corners" in g) == ("corners" in o), f"frame {t}: detection ran on one side only"
        if "corners" in g:
            gc, oc = g["corners"], o["corners"]
            assert (gc is None) == (oc is None), f"frame {t}: detection early exit differs"
            if gc is not None:
                assert np.array_equal(gc, oc), f"frame {t}: corners"
                n_detect += 1
        assert np.array_equal(pts, o["pts"]), f"frame {t}: track list"
    # the sequence exercised both halves of the loop
    assert n_tracked > 100 * (n_frames - 1) and n_detect >= 2


@pytest.mark.parametrize("graph,resident,pipeline,batch", [(False, False, False, 1), (True, False, False, 1),
                                                           (True, True, False, 1), (False, True, True, 1),
                                                           (True, True, True, 1), (False, True, True, 4),
                                                           (True, True, True, 4)])
def test_device_resident_sequence_matches(ctx, gvx_mod, graph, resident, pipeline, batch):
    """gvx_track_frame_dev (the tracker state on the device, no host round trip;
    with graph=True one captured graph per frame parity replayed per frame)
    gives the same per-frame track list as SequenceTracker, whose every step the
    test above holds bit-exact against the oracle.  pipeline: frame t+1's
    preprocessing runs as a side branch beside frame t's tracking (three frame
    slots; with graphs, a preprocessing graph and a tracking graph per slot
    rotation on two streams).  batch: K frames per preprocessing / tracking
    graph (3 sets of K slots)."""
    import torch
    from gvx import synth
    from gvx.tracking import DeviceSequenceTracker, SequenceTracker
    dev = torch.device("cuda", 0)
    n_frames = 30
    frames, _ = synth.make_sequence(W, H, n_frames, dev, seed=synth.SEED + 1)
    kp = gvx_mod.KltParams.default(max_level=L)
    dp = gvx_mod.DetectParams.default(max_features=N)
    ref = SequenceTracker(ctx, W, H, N, klt=kp, detect=dp, ids=(10, 11))
    trk = DeviceSequenceTracker(ctx, W, H, N, klt=kp, detect=dp, ids=(20, 21), graph=graph, device=dev,
                                frames=frames if resident else None, pipeline=pipeline, batch=batch)
    try:
        wants = []
        for t in range(n_frames):
            wants.append(ref.step(frames[t].data_ptr()))
            if resident:
                trk.step()  # the frame is picked on the device, nothing is read back per frame
                continue
            trk.step(frames[t].data_ptr())
            got = trk.tracks()
            assert np.array_equal(got, wants[t]), f"frame {t}: {got.shape} vs {wants[t].shape}"
        if resident:
            ctx.sync()
            counts = trk.rec_counts.cpu().numpy()
            tracks = trk.rec_tracks.cpu().numpy()
            assert int(trk.index.cpu()[0]) == n_frames
            for t in range(n_frames):
                assert np.array_equal(tracks[t, :counts[t]], wants[t]), f"frame {t}"
        if graph:
            assert len(trk.graphs) == (6 if pipeline else 2)
    finally:
        trk.close()


LONG = 300


@pytest.fixture(scope="module")
def long_sequence(orc, gvx_mod):
    """A 300-frame configs[4] sequence rendered on the device and the oracle's
    per-frame loop over it (host copy), computed once for the tests below."""
    import torch
    from gvx import synth
    dev = torch.device("cuda", 0)
    frames, _ = synth.make_sequence(W, H, LONG, dev, seed=synth.SEED + 2)
    ref = _oracle_sequence(orc, frames.cpu().numpy(), orc.KltParams.default(max_level=L), orc.DetectParams.default(),
                           nthreads=8)
    return frames, ref


def test_long_sequence_bit_exact(ctx, orc, gvx_mod, long_sequence):
    """300 frames of the host loop, every frame's forward /
    backward flow, status, keep flags, kept indices, detected corners and track
    list bit-exact against the oracle loop -- dozens of detection top-ups."""
    from gvx.tracking import SequenceTracker
    frames, ref = long_sequence
    tr = SequenceTracker(ctx, W, H, N, klt=gvx_mod.KltParams.default(max_level=L),
                         detect=gvx_mod.DetectParams.default(max_features=N), ids=(30, 31))
    n_detect = 0
    for t in range(LONG):
        pts = tr.step(frames[t].data_ptr())
        g, o = tr.last, ref[t]
        assert ("track" in g) == ("track" in o), f"frame {t}: tracking ran on one side only"
        if "track" in g:
            for k in ("next", "back", "st_f", "st_b", "keep", "kept_idx"):
                assert np.array_equal(g["track"][k], o["track"][k]), f"frame {t}: {k}"
        assert ("corners" in g) == ("corners" in o), f"frame {t}: detection ran on one side only"
        if "corners" in g and g["corners"] is not None:
            assert np.array_equal(g["corners"], o["corners"]), f"frame {t}: corners"
            n_detect += g["corners"].shape[0] > 0
        assert np.array_equal(pts, o["pts"]), f"frame {t}: track list"
    assert n_detect >= 10, n_detect


@pytest.mark.parametrize("pipeline,eig_branch,batch", [(False, False, 1), (True, False, 1), (True, True, 1),
                                                       (True, False, 8), (True, True, 7), (True, False, 16)])
def test_long_sequence_graph_replay(ctx, gvx_mod, long_sequence, pipeline, eig_branch, batch):
    """The bench's loop over the same 300 frames: the HBM-resident sequence, one
    captured graph per frame-slot rotation replayed per frame (pipelined: frame
    t+1's CLAHE + pyramid graph on the side stream beside frame t's tracking
    graph, three slots rotating 100 times), the per-frame track records written
    on the device -- every record bit-exact against the oracle loop's track list.
    eig_branch: the detection's eigenvalue maps computed on the preprocessing
    branch (gvx_frame_eig_dev) instead of in the tracking graph.  batch: K frames
    per graph (the bench's configs[4] loop); 300 = 42 x 7 + 6 ends on a short
    eager batch."""
    from gvx.tracking import DeviceSequenceTracker
    frames, ref = long_sequence
    trk = DeviceSequenceTracker(ctx, W, H, N, klt=gvx_mod.KltParams.default(max_level=L),
                                detect=gvx_mod.DetectParams.default(max_features=N), ids=(40, 41), graph=True,
                                frames=frames, pipeline=pipeline, eig_branch=eig_branch, batch=batch)
    try:
        for _ in range(LONG):
            trk.step()
        with pytest.raises(IndexError):
            trk.step()  # past the resident sequence
        ctx.sync()
        assert int(trk.index.cpu()[0]) == LONG
        counts = trk.rec_counts.cpu().numpy()
        tracks = trk.rec_tracks.cpu().numpy()
        for t in range(LONG):
            assert np.array_equal(tracks[t, :counts[t]], ref[t]["pts"]), f"frame {t}"
        assert len(trk.graphs) == (6 if pipeline else 2)
    finally:
        trk.close()


def test_partly_flat_frames_match_oracle(ctx, orc, gvx_mod):
    """Frames whose left half is flat for a while: the blocks there have an
    eigenvalue maximum of 0, so the tracking path's selection takes its full-ROI
    scan (the tiles' candidate lists only hold for a maximum > 0) while the
    textured blocks use the lists -- every frame's track list bit-exact against
    the oracle loop."""
    import torch
    from gvx import synth
    from gvx.tracking import DeviceSequenceTracker
    dev = torch.device("cuda", 0)
    n = 12
    frames, _ = synth.make_sequence(W, H, n, dev, seed=synth.SEED + 3)
    frames[4:8, :, :W // 2] = 128
    ref = _oracle_sequence(orc, frames.cpu().numpy(), orc.KltParams.default(max_level=L), orc.DetectParams.default(),
                           nthreads=8)
    trk = DeviceSequenceTracker(ctx, W, H, N, klt=gvx_mod.KltParams.default(max_level=L),
                                detect=gvx_mod.DetectParams.default(max_features=N), ids=(50, 51), graph=False,
                                device=dev, frames=frames)
    try:
        for _ in range(n):
            trk.step()
        ctx.sync()
        counts = trk.rec_counts.cpu().numpy()
        tracks = trk.rec_tracks.cpu().numpy()
        for t in range(n):
            assert np.array_equal(tracks[t, :counts[t]], ref[t]["pts"]), f"frame {t}"
        # the flat half lost its points and was detected on again
        assert any("corners" in ref[t] for t in range(4, 9))
    finally:
        trk.close()
