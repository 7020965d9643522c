// api_track.cpp -- gvx_track_frame_dev: one frame of Tracking::track's image
// path (tracking/tracking.cc:144-245 without the IMU parts) with the tracker
// state in device memory: forward + backward LK of the tracked points on two
// cached frames, the FB / border / status filter and reduceVector, then the
// block-grid detection topping the tracks up to track_max_features_.  No
// host round trip: every count lives on the device (kernels in klt.hip,
// detect.hip and track.hip), so the call is capturable into a hipGraph once the
// scratch buffers and the detection constants exist (one uncaptured call).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <vector>

#include "gvx_internal.h"

using namespace gvx;

namespace {

// The detection geometry of a W x H frame (Tracking ctor block grid,
// tracking.cc:65-85, as gvx_detect) and its device constants (block ROIs,
// circle half-widths, cornerSubPix weights), uploaded when the geometry
// changes -- never inside a capture.
struct DetGeom {
    int bcols, brows, bcnt, row, col, maxpb, mindist, mpb;
    int64_t stride;  // eig / candidate floats per block
    int4* rois;
    int* hw;
    float* gm;
    float sc, sc2;   // Sobel scale 1/(4*3*255) and 2x
    long key() const { return ((long)bcols * 4096 + brows) * 65536 + maxpb * 256 + mindist + 1; }
};

gvx_status det_geometry(gvx_ctx* c, int W, int H, const gvx_detect_params* dp, DetGeom* G) {
    DetGeom& g = *G;
    g.bcols = (int)std::lround(W / dp->block_size);
    g.brows = (int)std::lround(H / dp->block_size);
    g.bcnt = g.bcols * g.brows;
    if (g.bcols <= 0 || g.brows <= 0 || g.bcnt > 1024) return set_err(c, GVX_ERR_INVALID, "block grid %dx%d", g.bcols, g.brows);
    g.row = H / g.brows;
    g.col = W / g.bcols;
    g.maxpb = (int)std::lround((double)dp->max_features / (double)g.bcnt);
    g.mindist = g.maxpb > 0 ? (int)std::round(dp->block_size / std::sqrt(g.maxpb * 1.5)) : 0;
    g.stride = (int64_t)g.col * g.row;
    g.mpb = g.maxpb > 0 ? g.maxpb : 1;
    double sc = (double)(1 << (3 - 1)) * 3;
    sc *= 255.0;
    sc = 1.0 / sc;
    g.sc = (float)sc;
    g.sc2 = (float)(2.0 * sc);
    Staging st;
    st.add((size_t)g.bcnt, &g.rois);
    st.add((size_t)g.mindist + 1, &g.hw);
    st.add(121, &g.gm);
    void* sb = scratch(c, "trk_static", st.bytes());
    if (!sb) return set_err(c, GVX_ERR_OOM, "track constants");
    st.bind(sb);
    gvx_ctx::TrackStatic key;
    key.buf = sb;
    key.bytes = st.bytes();
    key.w = W;
    key.h = H;
    key.max_features = dp->max_features;
    key.block_size = std::lround(dp->block_size);
    if (!(c->track_static == key)) {
        if (c->capturing) {
            c->capture_failed = true;
            return set_err(c, GVX_ERR_INVALID, "detection constants not uploaded before the capture");
        }
        std::vector<int4> r(g.bcnt);
        for (int k = 0; k < g.bcnt; ++k) {
            const int bc = k % g.bcols, br = k / g.bcols;
            int cs = bc * g.col, ce = cs + g.col, rs = br * g.row, re = rs + g.row;
            if (k != g.bcnt - 1) {
                ce -= 5;
                re -= 5;
            }
            r[k] = make_int4(cs, rs, ce - cs, re - rs);
        }
        std::vector<int> h(g.mindist + 1, -1);
        {
            int err = 0, dx = g.mindist, dy = 0, plus = 1, minus = (g.mindist << 1) - 1;
            while (dx >= dy) {
                if (dy <= g.mindist) h[dy] = std::max(h[dy], dx);
                if (dx <= g.mindist) h[dx] = std::max(h[dx], dy);
                dy++;
                err += plus;
                plus += 2;
                const int m = (err <= 0) - 1;
                err -= minus & m;
                dx += m;
                minus -= m & 2;
            }
        }
        float gw[121];
        for (int i = 0; i < 11; ++i) {
            const float y = (float)(i - 5) / 5;
            const float vy = std::exp(-y * y);
            for (int j = 0; j < 11; ++j) {
                const float x = (float)(j - 5) / 5;
                gw[i * 11 + j] = (float)(vy * std::exp(-x * x));
            }
        }
        hipError_t e = hipMemcpyAsync(g.rois, r.data(), sizeof(int4) * g.bcnt, hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(g.hw, h.data(), sizeof(int) * h.size(), hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(g.gm, gw, sizeof gw, hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);  // pageable sources
        if (e != hipSuccess) return hip_err(c, e, "track constants upload");
        c->track_static = key;
    }
    return GVX_OK;
}

}  // namespace

// cornerMinEigenVal of every detection block of frame id into the frame's own
// eigenvalue map (kept until the frame is written again); the tracking call
// on this frame then skips that launch.
extern "C" gvx_status gvx_frame_eig_dev(gvx_ctx* c, uint64_t id, const gvx_detect_params* dp) {
    if (!c || !dp) return GVX_ERR_INVALID;
    auto it = c->frames.find(id);
    if (it == c->frames.end()) return set_err(c, GVX_ERR_NOT_FOUND, "frame %llu", (unsigned long long)id);
    Frame& f = it->second;
    hipSetDevice(c->device);
    DetGeom g{};
    gvx_status s = det_geometry(c, f.w, f.h, dp, &g);
    if (s) return s;
    const size_t bytes = sizeof(float) * (size_t)g.stride * g.bcnt;
    if (!f.eig || f.eig_bytes < bytes) {
        if (c->capturing) {
            c->capture_failed = true;
            return set_err(c, GVX_ERR_INVALID, "frame %llu's eigenvalue map needs an allocation during a capture",
                           (unsigned long long)id);
        }
        ++c->mem_gen;
        if (f.eig) {
            sync_all(c);
            hipFree(f.eig);
            f.eig = nullptr;
        }
        hipError_t e = hipMalloc(&f.eig, bytes);
        if (e != hipSuccess) return hip_err(c, e, "hipMalloc(eigenvalue map)");
        f.eig_bytes = bytes;
    }
    const int pitch = f.lay.pitch[0];
    const uint8_t* img0 = f.pyr + f.lay.off[0] + (int64_t)PAD * pitch + PAD;
    hipEvent_t ev{};
    prof_begin(c, "detect", &ev);
    hipError_t e = launch_eig_all(c, g.bcnt, g.col, g.row, img0, pitch, g.rois, g.stride, f.eig, g.sc, g.sc2);
    prof_end(c, "detect", ev);
    if (e != hipSuccess) return hip_err(c, e, "eigenvalue tiles");
    f.eig_key = g.key();
    f.eig_gen = f.gen;
    return GVX_OK;
}

static gvx_status track_frame(gvx_ctx* c, uint64_t prev_id, uint64_t next_id, int32_t track, float* d_pts,
                              float* d_vel, float* d_init, int32_t* d_n, int32_t cap, int32_t cam_w, int32_t cam_h,
                              double fb_thresh, double border, const gvx_klt_params* kp, const gvx_detect_params* dp,
                              int32_t* d_kept, float* d_corners, int32_t* d_n_corners, const TrackRecord* rec) {
    if (!c || !kp || !dp) return GVX_ERR_INVALID;
    if (!d_pts || !d_vel || !d_init || !d_n) return set_err(c, GVX_ERR_INVALID, "null tracker state");
    if (cap <= 0 || cap < dp->max_features) return set_err(c, GVX_ERR_INVALID, "capacity %d < max_features", cap);
    if (kp->win != WIN) return set_err(c, GVX_ERR_UNSUPPORTED, "device LK supports win=21 only (got %d)", kp->win);
    if (kp->accum < GVX_LK_ACCUM_EXACT || kp->accum > GVX_LK_ACCUM_F32_SIMD4)
        return set_err(c, GVX_ERR_INVALID, "unknown LK accumulation order %d", kp->accum);
    if (dp->subpix_win != 5) return set_err(c, GVX_ERR_UNSUPPORTED, "cornerSubPix win must be 5 (tracking.cc:623)");
    auto in = c->frames.find(next_id);
    if (in == c->frames.end()) return set_err(c, GVX_ERR_NOT_FOUND, "frame %llu", (unsigned long long)next_id);
    const Frame& fn = in->second;
    const int W = fn.w, H = fn.h;
    const Frame* fp = nullptr;
    if (track) {
        auto ip = c->frames.find(prev_id);
        if (ip == c->frames.end()) return set_err(c, GVX_ERR_NOT_FOUND, "frame %llu", (unsigned long long)prev_id);
        fp = &ip->second;
        if (fp->w != W || fp->h != H) return set_err(c, GVX_ERR_INVALID, "frame sizes differ");
    }
    DetGeom G{};
    gvx_status gs = det_geometry(c, W, H, dp, &G);
    if (gs) return gs;
    const int bcols = G.bcols, brows = G.brows, bcnt = G.bcnt, row = G.row, col = G.col, maxpb = G.maxpb;
    const int mindist = G.mindist, mpb = G.mpb;
    const int64_t stride = G.stride;
    int4* rois = G.rois;
    int* hw = G.hw;
    float* gm = G.gm;
    // the one-launch-per-block selection (select_track_kernel) where its LDS holds
    // the tracker and the ROI bitmap; the prep / mask / select form otherwise
    const bool fused = cap <= TS_MAX_POINTS && select_track_lds(col, row) <= TS_MAX_BITMAP;
    // the frame's own eigenvalue map when gvx_frame_eig_dev computed it for this image
    const bool pre_eig = fused && fn.eig && fn.eig_gen == fn.gen && fn.eig_key == G.key();
    hipSetDevice(c->device);
    // scratch: LK flags, detection buffers, the counts
    uint8_t *flags, *mask;
    int2 *cent, *corn;
    int *want, *ids, *nact, *ncirc, *skip, *nc;
    float* eig;
    unsigned long long* cand;
    float2* out;
    Staging st;
    st.add((size_t)cap, &flags);
    st.add((size_t)cap, &cent);
    st.add((size_t)bcnt, &want);
    st.add((size_t)bcnt, &ids);
    st.add(1, &nact);
    st.add(1, &ncirc);
    st.add(1, &skip);
    st.add(fused ? 0 : (size_t)W * H, &mask);
    st.add((size_t)stride * bcnt, &eig);
    st.add((size_t)stride * bcnt, &cand);
    st.add((size_t)mpb * bcnt, &corn);
    st.add((size_t)bcnt, &nc);
    st.add((size_t)mpb * bcnt, &out);
    void* db = scratch(c, "trk", st.bytes());
    if (!db) return set_err(c, GVX_ERR_OOM, "track scratch");
    st.bind(db);
    hipEvent_t ev{};
    hipError_t e = hipSuccess;
    if (track) {
        PyrLayout lay = fp->lay;
        lay.nlev = make_layout(W, H, kp->max_level, kp->win).nlev;
        if (lay.nlev > fp->lay.nlev || lay.nlev > fn.lay.nlev)
            return set_err(c, GVX_ERR_INVALID, "frames were put with a smaller max_level");
        KltArgs a{};
        int it = kp->max_iter;
        a.max_iter = it < 0 ? 0 : (it > 100 ? 100 : it);
        const double ce = kp->eps < 0 ? 0.0 : (kp->eps > 10.0 ? 10.0 : kp->eps);
        a.crit_eps = ce * ce;
        a.min_eig = kp->min_eig;
        a.accum = kp->accum;
        a.use_initial_flow = 1;  // pts + vel, as SequenceTracker / Tracking::track
        a.n_pairs = 1;
        a.n_pts = cap;
        a.n_dev = d_n;
        a.mode = 1;
        a.fb_thresh = fb_thresh;
        a.border = border;
        a.cam_w = cam_w;
        a.cam_h = cam_h;
        const Level0 l0{fp->pyr + lay.off[0], fn.pyr + lay.off[0], 0, 0, PAD * lay.pitch[0] + PAD, lay.pitch[0], 0};
        // d_init is the initial flow in and the tracked positions out
        e = launch_klt(c, a, lay, fp->pyr, fn.pyr, 0, 0, l0, d_pts, d_init, nullptr, flags, nullptr);
        if (e != hipSuccess) return hip_err(c, e, "klt kernel");
    }
    if (fused) {
        // one workgroup per block (counts, early exit, LDS circle mask, selection,
        // cornerSubPix), then the merge launch (FB update, corners, record)
        prof_begin(c, "detect", &ev);
        {
            TrackSelect ts{};
            ts.bcols = bcols;
            ts.col = col;
            ts.row = row;
            ts.maxpb = maxpb;
            ts.max_features = dp->max_features;
            ts.cap = cap;
            ts.radius = mindist;
            ts.n = d_n;
            ts.flags = track ? flags : nullptr;
            ts.next_xy = d_init;
            ts.pts = d_pts;
            ts.rois = rois;
            ts.hw = hw;
            ts.eig = pre_eig ? fn.eig : eig;
            ts.eig_stride = stride;
            ts.cand = cand;
            ts.corners = corn;
            ts.ncorner = nc;
            ts.max_per_block = mpb;
            ts.quality = dp->quality;
            ts.min_dist = (float)mindist;
            ts.pitch = fn.lay.pitch[0];
            ts.img0 = fn.pyr + fn.lay.off[0] + (int64_t)PAD * ts.pitch + PAD;
            ts.gmask = gm;
            ts.max_iters = dp->subpix_iters < 1 ? 1 : (dp->subpix_iters > 100 ? 100 : dp->subpix_iters);
            const double eps = dp->subpix_eps > 0 ? dp->subpix_eps : 0.0;
            ts.eps2 = eps * eps;
            ts.out = out;
            ts.sel = nullptr;
            if (!pre_eig) {
                // the tiles' max / candidate counters: zero once at allocation, then
                // cleared by the selection after each frame
                DevBuf& sb = c->dev["trk_sel"];
                ts.sel = (unsigned*)scratch(c, "trk_sel", (size_t)2 * bcnt * sizeof(unsigned));
                if (!ts.sel) return set_err(c, GVX_ERR_OOM, "selection counters");
                if (sb.fresh) {
                    e = hipMemsetAsync(sb.p, 0, sb.bytes, c->stream);
                    if (e != hipSuccess) return hip_err(c, e, "selection counters");
                    sb.fresh = false;
                }
            }
            // the eigenvalue tiles of the blocks that detect (unless the frame has its map)
            if (!pre_eig) e = launch_eig_track(c, bcnt, col, row, ts, G.sc, G.sc2);
            if (e == hipSuccess) e = launch_select_track(c, bcnt, col, row, ts);
        }
        if (e == hipSuccess) {
            TrackMerge m{};
            m.bcnt = bcnt;
            m.bcols = bcols;
            m.col = col;
            m.row = row;
            m.maxpb = maxpb;
            m.out_stride = mpb;
            m.max_features = dp->max_features;
            m.update_cap = track ? cap : 0;
            m.flags = flags;
            m.next_xy = d_init;
            m.pts = d_pts;
            m.vel = d_vel;
            m.init = d_init;
            m.kept_out = d_kept;
            m.n = d_n;
            m.ncorner = nc;
            m.out = out;
            m.corners_out = d_corners;
            m.n_corners_out = d_n_corners;
            if (rec) m.rec = *rec;
            e = launch_track_merge(c, m);
        }
        prof_end(c, "detect", ev);
        return hip_err(c, e, "detection kernels");
    }
    // reduceVector of the FB result (track frames) and the detection's counts /
    // circle centres: one single-workgroup launch
    DetectPrep pp{};
    if (track) {
        pp.update_cap = cap;
        pp.flags = flags;
        pp.next_xy = d_init;
        pp.upd_pts = d_pts;
        pp.vel = d_vel;
        pp.init = d_init;
        pp.kept_out = d_kept;
        pp.n_upd = d_n;
    }
    pp.bcols = bcols;
    pp.brows = brows;
    pp.col = col;
    pp.row = row;
    pp.maxpb = maxpb;
    pp.max_features = dp->max_features;
    pp.pts = d_pts;
    pp.n = d_n;
    pp.want = want;
    pp.blk_ids = ids;
    pp.n_active = nact;
    pp.centers = cent;
    pp.n_circles = ncirc;
    pp.skip = skip;
    pp.ncorner = nc;
    prof_begin(c, "detect", &ev);
    e = launch_detect_prep(c, pp);
    if (e == hipSuccess) {
        DetectLaunch d{};
        d.w = W;
        d.h = H;
        d.pitch = fn.lay.pitch[0];
        d.img0 = fn.pyr + fn.lay.off[0] + (int64_t)PAD * d.pitch + PAD;
        d.centers = cent;
        d.n_circles = 0;
        d.radius = mindist;
        d.fill_mask = 1;
        d.hw = hw;
        d.mask = mask;
        d.rois = rois;
        d.blk_ids = ids;
        d.n_active = 0;
        d.n_blocks = bcnt;
        d.max_rw = col;
        d.max_rh = row;
        d.want = want;
        d.eig_stride = stride;
        d.eig = eig;
        d.cand = cand;
        d.corners = corn;
        d.ncorner = nc;
        d.max_per_block = mpb;
        d.quality = dp->quality;
        d.min_dist = (float)mindist;
        double s = (double)(1 << (3 - 1)) * 3;
        s *= 255.0;
        s = 1.0 / s;
        d.sc = (float)s;
        d.sc2 = (float)(2.0 * s);
        d.gmask = gm;
        d.max_iters = dp->subpix_iters < 1 ? 1 : (dp->subpix_iters > 100 ? 100 : dp->subpix_iters);
        const double eps = dp->subpix_eps > 0 ? dp->subpix_eps : 0.0;
        d.eps2 = eps * eps;
        d.out = out;
        d.n_circles_dev = ncirc;
        d.n_active_dev = nact;
        d.skip_dev = skip;
        e = launch_detect(c, d);
    }
    if (e == hipSuccess)
        e = launch_detect_merge(c, bcnt, bcols, col, row, mpb, dp->max_features, skip, nc, out, d_pts, d_vel, d_init,
                                d_n, d_corners, d_n_corners, rec);
    prof_end(c, "detect", ev);
    return hip_err(c, e, "detection kernels");
}

extern "C" gvx_status gvx_track_frame_dev(gvx_ctx* c, uint64_t prev_id, uint64_t next_id, int32_t track,
                                          float* d_pts, float* d_vel, float* d_init, int32_t* d_n, int32_t cap,
                                          int32_t cam_w, int32_t cam_h, double fb_thresh, double border,
                                          const gvx_klt_params* kp, const gvx_detect_params* dp, int32_t* d_kept,
                                          float* d_corners, int32_t* d_n_corners) {
    return track_frame(c, prev_id, next_id, track, d_pts, d_vel, d_init, d_n, cap, cam_w, cam_h, fb_thresh, border,
                       kp, dp, d_kept, d_corners, d_n_corners, nullptr);
}

extern "C" gvx_status gvx_track_frame_record_dev(gvx_ctx* c, uint64_t prev_id, uint64_t next_id, int32_t track,
                                                 float* d_pts, float* d_vel, float* d_init, int32_t* d_n, int32_t cap,
                                                 int32_t cam_w, int32_t cam_h, double fb_thresh, double border,
                                                 const gvx_klt_params* kp, const gvx_detect_params* dp,
                                                 float* d_tracks, int32_t* d_counts, int32_t* d_frame_index,
                                                 int32_t max_frames) {
    if (!c) return GVX_ERR_INVALID;
    if (!d_tracks || !d_counts || !d_frame_index || max_frames < 0)
        return set_err(c, GVX_ERR_INVALID, "bad record arguments");
    const TrackRecord rec{d_tracks, d_counts, d_frame_index, max_frames, cap};
    return track_frame(c, prev_id, next_id, track, d_pts, d_vel, d_init, d_n, cap, cam_w, cam_h, fb_thresh, border,
                       kp, dp, nullptr, nullptr, nullptr, &rec);
}

extern "C" gvx_status gvx_copy_indexed_dev(gvx_ctx* c, void* d_dst, const void* d_src_base, size_t bytes,
                                           const int32_t* d_index, int32_t n_src) {
    if (!c) return GVX_ERR_INVALID;
    if (bytes == 0) return GVX_OK;
    if (!d_dst || !d_src_base || !d_index) return set_err(c, GVX_ERR_INVALID, "null device pointer");
    if (n_src <= 0) return set_err(c, GVX_ERR_INVALID, "n_src must be positive");
    hipSetDevice(c->device);
    return hip_err(c, launch_copy_indexed(c, d_dst, d_src_base, bytes, d_index, n_src), "indexed copy kernel");
}

extern "C" gvx_status gvx_track_record_dev(gvx_ctx* c, const float* d_pts, const int32_t* d_n, int32_t capacity,
                                           float* d_tracks, int32_t* d_counts, int32_t* d_frame_index,
                                           int32_t max_frames) {
    if (!c) return GVX_ERR_INVALID;
    if (!d_pts || !d_n || !d_tracks || !d_counts || !d_frame_index || capacity <= 0 || max_frames < 0)
        return set_err(c, GVX_ERR_INVALID, "bad record arguments");
    hipSetDevice(c->device);
    return hip_err(c, launch_track_record(c, d_pts, d_n, capacity, d_tracks, d_counts, d_frame_index, max_frames),
                   "track record kernel");
}

gvx_status gvx_index_advance_dev(gvx_ctx* c, int32_t* d_index, int32_t delta) {
    if (!c) return GVX_ERR_INVALID;
    if (!d_index) return set_err(c, GVX_ERR_INVALID, "null device pointer");
    hipSetDevice(c->device);
    return hip_err(c, launch_index_advance(c, d_index, delta), "index advance kernel");
}
