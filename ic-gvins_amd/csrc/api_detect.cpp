// api_detect.cpp -- gvx_detect: Tracking::featuresDetection
// (/root/reference/ic_gvins/ic_gvins/tracking/tracking.cc:576-688) on a cached frame.
// Host side: block grid (Tracking ctor, tracking.cc:65-85), per-block existing
// feature counts (:585-606), circle centres and the cornerSubPix weight mask;
// device side: detect.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <vector>

#include "gvx_internal.h"

using namespace gvx;

extern "C" {

void gvx_detect_params_default(gvx_detect_params* p) {
    if (!p) return;
    p->block_size = 200.0;
    p->max_features = 150;
    p->quality = 0.01;
    p->subpix_win = 5;
    p->subpix_iters = 20;
    p->subpix_eps = 0.01;
}

gvx_status gvx_detect(gvx_ctx* c, uint64_t frame_id, const float* count_xy, int32_t n_count,
                      const float* mask_xy, int32_t n_mask, int32_t ismask, int32_t n_existing,
                      const gvx_detect_params* p, float* out_xy, int32_t* out_block_counts, int32_t* n_out) {
    if (!c || !p || !n_out) return GVX_ERR_INVALID;
    if (p->subpix_win != 5) return set_err(c, GVX_ERR_UNSUPPORTED, "cornerSubPix win must be 5 (tracking.cc:623)");
    if (n_count < 0 || n_mask < 0 || (n_count && !count_xy) || (ismask && n_mask && !mask_xy))
        return set_err(c, GVX_ERR_INVALID, "bad point lists");
    auto it = c->frames.find(frame_id);
    if (it == c->frames.end()) return set_err(c, GVX_ERR_NOT_FOUND, "frame %llu", (unsigned long long)frame_id);
    const Frame& f = it->second;
    const int W = f.w, H = f.h;
    // Tracking ctor block grid
    const int bcols = (int)std::lround(W / p->block_size);
    const int brows = (int)std::lround(H / p->block_size);
    const int bcnt = bcols * brows;
    if (bcols <= 0 || brows <= 0) return set_err(c, GVX_ERR_INVALID, "image smaller than half a block");
    const int row = H / brows, col = W / bcols;
    const int maxpb = (int)std::lround((double)p->max_features / (double)bcnt);
    const int mindist = (int)std::round(p->block_size / std::sqrt(maxpb * 1.5));
    if (out_block_counts) std::memset(out_block_counts, 0, sizeof(int32_t) * bcnt);
    if (n_existing > p->max_features - 5) {
        *n_out = -1;
        return GVX_OK;
    }
    if (maxpb <= 0) {
        *n_out = 0;
        return GVX_OK;
    }
    if (!out_xy) return set_err(c, GVX_ERR_INVALID, "null out_xy");
    // existing features per block (flat index like the reference's VLA; out of
    // range indices -- undefined behaviour there -- are skipped)
    std::vector<int> cnt(bcnt, 0), want(bcnt, 0), active;
    for (int i = 0; i < n_count; ++i) {
        const int cc = (int)(count_xy[2 * i] / (float)col);
        const int rr = (int)(count_xy[2 * i + 1] / (float)row);
        const int idx = rr * bcols + cc;
        if (idx >= 0 && idx < bcnt) cnt[idx]++;
    }
    std::vector<int4> rois(bcnt);
    for (int k = 0; k < bcnt; ++k) {
        want[k] = maxpb - cnt[k];
        const int bc = k % bcols, br = k / bcols;
        int cs = bc * col, ce = cs + col, rs = br * row, re = rs + row;
        if (k != bcnt - 1) {
            ce -= 5;
            re -= 5;
        }
        rois[k] = make_int4(cs, rs, ce - cs, re - rs);
        if (want[k] > 0) active.push_back(k);
    }
    // circle centres: Point2f -> Point via cvRound (round half to even)
    std::vector<int2> centers;
    if (ismask)
        for (int i = 0; i < n_mask; ++i)
            centers.push_back(make_int2((int)std::lrintf(mask_xy[2 * i]), (int)std::lrintf(mask_xy[2 * i + 1])));
    // per-row half widths of Circle(..., fill) (imgproc/src/drawing.cpp midpoint loop)
    std::vector<int> hw(mindist + 1, -1);
    {
        int err = 0, dx = mindist, dy = 0, plus = 1, minus = (mindist << 1) - 1;
        while (dx >= dy) {
            if (dy <= mindist) hw[dy] = std::max(hw[dy], dx);
            if (dx <= mindist) hw[dx] = std::max(hw[dx], dy);
            dy++;
            err += plus;
            plus += 2;
            const int m = (err <= 0) - 1;
            err -= minus & m;
            dx += m;
            minus -= m & 2;
        }
    }
    // cornerSubPix weights (cornersubpix.cpp): float y = (i - win)/win; exp(-y*y)*exp(-x*x)
    float gmask[121];
    {
        const int win = 5;
        for (int i = 0; i < 11; ++i) {
            const float y = (float)(i - win) / win;
            const float vy = std::exp(-y * y);
            for (int j = 0; j < 11; ++j) {
                const float x = (float)(j - win) / win;
                gmask[i * 11 + j] = (float)(vy * std::exp(-x * x));
            }
        }
    }
    const int64_t stride = (int64_t)col * row;
    hipSetDevice(c->device);
    int2 *d_cent, *d_corn;
    int *d_hw, *d_ids, *d_want, *d_nc;
    int4* d_rois;
    uint8_t* d_mask;
    float *d_eig, *d_gm;
    unsigned long long* d_cand;
    float2* d_out;
    Staging st;
    st.add(centers.size() + 1, &d_cent);
    st.add((size_t)mindist + 1, &d_hw);
    st.add((size_t)bcnt, &d_rois);
    st.add(active.size() + 1, &d_ids);
    st.add((size_t)bcnt, &d_want);
    st.add((size_t)W * H, &d_mask);
    st.add((size_t)stride * bcnt, &d_eig);
    st.add((size_t)stride * bcnt, &d_cand);
    st.add((size_t)maxpb * bcnt, &d_corn);
    st.add((size_t)bcnt, &d_nc);
    st.add((size_t)maxpb * bcnt, &d_out);
    st.add(121, &d_gm);
    void* db = scratch(c, "detect", st.bytes());
    if (!db) return set_err(c, GVX_ERR_OOM, "detect staging");
    st.bind(db);
    hipError_t e = hipSuccess;
    auto up = [&](void* d, const void* h, size_t b) {
        if (e == hipSuccess && b) e = hipMemcpyAsync(d, h, b, hipMemcpyHostToDevice, c->stream);
    };
    // staging from pageable host memory: keep the host vectors alive until the sync below
    up(d_cent, centers.data(), sizeof(int2) * centers.size());
    up(d_hw, hw.data(), sizeof(int) * hw.size());
    up(d_rois, rois.data(), sizeof(int4) * bcnt);
    up(d_ids, active.data(), sizeof(int) * active.size());
    up(d_want, want.data(), sizeof(int) * bcnt);
    up(d_gm, gmask, sizeof(gmask));
    if (e == hipSuccess) e = hipMemsetAsync(d_nc, 0, sizeof(int) * bcnt, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "detect H2D");
    DetectLaunch d{};
    d.w = W;
    d.h = H;
    d.pitch = f.lay.pitch[0];
    d.img0 = f.pyr + f.lay.off[0] + (int64_t)PAD * d.pitch + PAD;
    d.centers = d_cent;
    d.n_circles = (int)centers.size();
    d.radius = mindist;
    d.fill_mask = 1;
    d.hw = d_hw;
    d.mask = d_mask;
    d.rois = d_rois;
    d.blk_ids = d_ids;
    d.n_active = (int)active.size();
    d.n_blocks = bcnt;
    d.max_rw = col;
    d.max_rh = row;
    d.want = d_want;
    d.eig_stride = stride;
    d.eig = d_eig;
    d.cand = d_cand;
    d.corners = d_corn;
    d.ncorner = d_nc;
    d.max_per_block = maxpb;
    d.quality = p->quality;
    d.min_dist = (float)mindist;
    {
        double scale = (double)(1 << (3 - 1)) * 3;
        scale *= 255.0;
        scale = 1.0 / scale;
        d.sc = (float)scale;
        d.sc2 = (float)(2.0 * scale);
    }
    d.gmask = d_gm;
    d.max_iters = p->subpix_iters < 1 ? 1 : (p->subpix_iters > 100 ? 100 : p->subpix_iters);
    const double eps = p->subpix_eps > 0 ? p->subpix_eps : 0.0;
    d.eps2 = eps * eps;
    d.out = d_out;
    hipEvent_t ev{};
    prof_begin(c, "detect", &ev);
    e = launch_detect(c, d);
    prof_end(c, "detect", ev);
    if (e != hipSuccess) return hip_err(c, e, "detect kernels");
    std::vector<int> nc(bcnt);
    std::vector<float2> outv((size_t)maxpb * bcnt);
    e = hipMemcpyAsync(nc.data(), d_nc, sizeof(int) * bcnt, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(outv.data(), d_out, sizeof(float2) * outv.size(), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "detect D2H");
    int total = 0;
    for (int k = 0; k < bcnt; ++k) {
        const int bc = k % bcols, br = k / bcols;
        for (int i = 0; i < nc[k]; ++i) {
            const float2 v = outv[(size_t)k * maxpb + i];
            out_xy[2 * total] = (float)(bc * col) + v.x;
            out_xy[2 * total + 1] = (float)(br * row) + v.y;
            ++total;
        }
        if (out_block_counts) out_block_counts[k] = nc[k];
    }
    *n_out = total;
    return GVX_OK;
}

}  // extern "C"
