// api_fmat.cpp -- C ABI of the device cv::findFundamentalMat(FM_RANSAC)
// (include/gvx.h; kernel in fmat.hip), the outlier rejection of
// Tracking::trackReferenceFrame (tracking/tracking.cc:547-555).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "gvx_internal.h"

using namespace gvx;

namespace {

gvx_status check_sets(gvx_ctx* c, int32_t n_sets, const int32_t* off) {
    if (n_sets < 0) return set_err(c, GVX_ERR_INVALID, "n_sets < 0");
    if (n_sets && !off) return set_err(c, GVX_ERR_INVALID, "null offsets");
    return GVX_OK;
}

}  // namespace

gvx_status gvx_find_fundamental_ransac_dev(gvx_ctx* c, int32_t n_sets, const int32_t* d_off, const float* d_p1,
                                           const float* d_p2, double thresh, double confidence, int32_t max_iters,
                                           uint8_t* d_mask, double* d_F, int32_t* d_result) {
    if (!c) return GVX_ERR_INVALID;
    gvx_status s = check_sets(c, n_sets, d_off);
    if (s) return s;
    if (n_sets == 0) return GVX_OK;
    if (!d_p1 || !d_p2 || !d_mask || !d_result) return set_err(c, GVX_ERR_INVALID, "null device pointer");
    hipSetDevice(c->device);
    hipEvent_t ev{};
    prof_begin(c, "fmat", &ev);
    hipError_t e = launch_fm_ransac(c, n_sets, d_off, d_p1, d_p2, thresh, confidence, max_iters, d_mask, d_F, d_result);
    prof_end(c, "fmat", ev);
    return hip_err(c, e, "findFundamentalMat kernel");
}

gvx_status gvx_find_fundamental_ransac(gvx_ctx* c, int32_t n_sets, const int32_t* off, const float* p1,
                                       const float* p2, double thresh, double confidence, int32_t max_iters,
                                       uint8_t* mask, double* F, int32_t* result) {
    if (!c) return GVX_ERR_INVALID;
    gvx_status s = check_sets(c, n_sets, off);
    if (s) return s;
    if (n_sets == 0) return GVX_OK;
    if (off[0] != 0) return set_err(c, GVX_ERR_INVALID, "off[0] != 0");
    for (int i = 0; i < n_sets; ++i)
        if (off[i + 1] < off[i]) return set_err(c, GVX_ERR_INVALID, "set %d: negative size", i);
    const int64_t n = off[n_sets];
    if (n && (!p1 || !p2 || !mask)) return set_err(c, GVX_ERR_INVALID, "null pointer");
    if (!result) return set_err(c, GVX_ERR_INVALID, "null result");
    hipSetDevice(c->device);
    int32_t *d_off, *h_off, *d_res, *h_res;
    float *d_p1, *h_p1, *d_p2, *h_p2;
    uint8_t *d_mask, *h_mask;
    double *d_F, *h_F;
    unsigned long long *d_ts, *h_ts;
    Staging st;
    st.add((size_t)n_sets + 1, &d_off, &h_off);
    st.add((size_t)n * 2, &d_p1, &h_p1);
    st.add((size_t)n * 2, &d_p2, &h_p2);
    st.add((size_t)n_sets, &d_res, &h_res);
    st.add((size_t)n, &d_mask, &h_mask);
    st.add((size_t)n_sets * 9, &d_F, &h_F);
    st.add(24, &d_ts, &h_ts);
    // GVX_FM_TIMING=1: per-phase times of the first set's first batches to stderr (diagnostics)
    static const bool timing = getenv("GVX_FM_TIMING") && *getenv("GVX_FM_TIMING") == '1';
    hipError_t e = hipStreamSynchronize(c->stream);  // the pinned arena may feed an earlier upload
    if (e != hipSuccess) return hip_err(c, e, "findFundamentalMat: stream");
    void* hb = pinned(c, "fmat", st.bytes());
    void* db = scratch(c, "fmat", st.bytes());
    if (!hb || !db) return set_err(c, GVX_ERR_OOM, "findFundamentalMat staging");
    st.bind(db, hb);
    std::memcpy(h_off, off, sizeof(int32_t) * (n_sets + 1));
    if (n) {
        std::memcpy(h_p1, p1, sizeof(float) * 2 * n);
        std::memcpy(h_p2, p2, sizeof(float) * 2 * n);
    }
    e = hipMemcpyAsync(d_off, h_off, (size_t)((char*)d_res - (char*)d_off), hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "findFundamentalMat upload");
    if (timing) {
        e = launch_fm_ransac(c, n_sets, d_off, d_p1, d_p2, thresh, confidence, max_iters, d_mask, d_F, d_res, d_ts);
        if (e != hipSuccess) return hip_err(c, e, "findFundamentalMat kernel");
    } else {
        s = gvx_find_fundamental_ransac_dev(c, n_sets, d_off, d_p1, d_p2, thresh, confidence, max_iters, d_mask, d_F,
                                            d_res);
        if (s) return s;
    }
    e = hipMemcpyAsync(h_res, d_res, (size_t)((char*)(d_ts + 24) - (char*)d_res),
                       hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "findFundamentalMat download");
    std::memcpy(result, h_res, sizeof(int32_t) * n_sets);
    if (n) std::memcpy(mask, h_mask, (size_t)n);
    if (F) std::memcpy(F, h_F, sizeof(double) * 9 * n_sets);
    if (timing)
        for (unsigned long long b = 0; b < h_ts[20] && b < 4; ++b)
            fprintf(stderr, "gvx fmat batch %llu us: subsets %.1f run7point %.1f counts %.1f replay %.1f\n", b,
                    (h_ts[b * 5 + 1] - h_ts[b * 5]) * 0.01, (h_ts[b * 5 + 2] - h_ts[b * 5 + 1]) * 0.01,
                    (h_ts[b * 5 + 3] - h_ts[b * 5 + 2]) * 0.01, (h_ts[b * 5 + 4] - h_ts[b * 5 + 3]) * 0.01);
    return GVX_OK;
}
