// api_clahe.cpp -- C ABI of the preprocessing step (include/gvx.h):
// Tracking::preprocessing (/root/reference/ic_gvins/ic_gvins/tracking/tracking.cc:107-141).
#include <cmath>
#include <cstring>

#include "gvx_internal.h"

using namespace gvx;

void gvx_clahe_params_default(gvx_clahe_params* p) {
    if (!p) return;
    p->clip_limit = 3.0;  // cv::createCLAHE(3.0, cv::Size(21, 21)), tracking.cc:63
    p->tiles_x = 21;
    p->tiles_y = 21;
    p->channels = 1;
}

// bytes per pixel of the source frame (gvx_clahe_params.channels; validated)
static int chan_of(const gvx_clahe_params* cp) { return cp && cp->channels == 3 ? 3 : 1; }

static gvx_status check_clahe(gvx_ctx* c, int w, int h, const gvx_clahe_params* cp) {
    if (!cp) return set_err(c, GVX_ERR_INVALID, "null CLAHE params");
    if (cp->channels != 1 && cp->channels != 3)
        return set_err(c, GVX_ERR_INVALID, "source channels %d (1 = MONO8, 3 = BGR8)", cp->channels);
    if (cp->tiles_x < 1 || cp->tiles_y < 1 || cp->tiles_x > GVX_CLAHE_MAX_TILES || cp->tiles_y > GVX_CLAHE_MAX_TILES)
        return set_err(c, GVX_ERR_INVALID, "CLAHE tile grid %dx%d outside [1, %d]", cp->tiles_x, cp->tiles_y,
                       GVX_CLAHE_MAX_TILES);
    if (!std::isfinite(cp->clip_limit)) return set_err(c, GVX_ERR_INVALID, "CLAHE clip limit not finite");
    // copyMakeBorder(REFLECT_101) of up to tiles-1 pixels needs tiles <= size
    if (w < cp->tiles_x || h < cp->tiles_y)
        return set_err(c, GVX_ERR_INVALID, "image %dx%d smaller than the CLAHE tile grid", w, h);
    return GVX_OK;
}

// Enqueue CLAHE (and the histogram means when d_mean) on the context stream.
static gvx_status clahe_enqueue(gvx_ctx* c, int n, int w, int h, const uint8_t* src, int64_t img_stride,
                                int stride, uint8_t* dst, int64_t dst_img_stride, int dst_stride,
                                const gvx_clahe_params* cp, double* d_mean, const int32_t* src_index = nullptr,
                                int n_src = 0, int ring = 0) {
    const ClaheGeom g = clahe_geometry(w, h, cp->clip_limit, cp->tiles_x, cp->tiles_y);
    uint8_t* lut = (uint8_t*)scratch(c, "clahe_lut", (size_t)n * g.tiles_x * g.tiles_y * 256);
    uint32_t* hist = d_mean ? (uint32_t*)scratch(c, "clahe_hist", (size_t)n * 256 * sizeof(uint32_t)) : nullptr;
    const int chan = chan_of(cp);
    uint8_t* gray = chan == 3 ? (uint8_t*)scratch(c, "clahe_gray", (size_t)n * clahe_gray_pitch(w) * h) : nullptr;
    if (!lut || (d_mean && !hist) || (chan == 3 && !gray)) return set_err(c, GVX_ERR_OOM, "CLAHE scratch");
    hipEvent_t ev{};
    prof_begin(c, "clahe", &ev);
    hipError_t e = launch_clahe(c, n, g, src, img_stride, stride, dst, dst_img_stride, dst_stride, lut, hist, d_mean,
                                src_index, n_src, ring, chan, gray);
    prof_end(c, "clahe", ev);
    return hip_err(c, e, "CLAHE kernels");
}

gvx_status gvx_clahe_batch_dev(gvx_ctx* c, int32_t n, int32_t w, int32_t h, const uint8_t* d_src,
                               int64_t src_img_stride, int32_t src_stride, uint8_t* d_dst,
                               int64_t dst_img_stride, int32_t dst_stride, const gvx_clahe_params* cp,
                               double* d_hist_mean) {
    if (!c) return GVX_ERR_INVALID;
    const int ch = chan_of(cp);
    if (n < 0 || w <= 0 || h <= 0 || src_stride < ch * w || dst_stride < w || (n > 0 && (!d_src || !d_dst)))
        return set_err(c, GVX_ERR_INVALID, "bad CLAHE batch");
    if (n > 1 && (src_img_stride < (int64_t)src_stride * h || dst_img_stride < (int64_t)dst_stride * h))
        return set_err(c, GVX_ERR_INVALID, "CLAHE image strides overlap");
    gvx_status s = check_clahe(c, w, h, cp);
    if (s || n == 0) return s;
    hipSetDevice(c->device);
    return clahe_enqueue(c, n, w, h, d_src, src_img_stride, src_stride, d_dst, dst_img_stride, dst_stride, cp,
                         d_hist_mean);
}

gvx_status gvx_clahe(gvx_ctx* c, int32_t w, int32_t h, const uint8_t* src, int32_t src_stride, uint8_t* dst,
                     int32_t dst_stride, const gvx_clahe_params* cp, double* hist_mean) {
    if (!c) return GVX_ERR_INVALID;
    const int ch = chan_of(cp);
    if (!src || !dst || w <= 0 || h <= 0 || src_stride < ch * w || dst_stride < w)
        return set_err(c, GVX_ERR_INVALID, "bad CLAHE image");
    gvx_status s = check_clahe(c, w, h, cp);
    if (s) return s;
    hipSetDevice(c->device);
    const size_t nb = (size_t)w * h, nin = nb * ch;
    uint8_t* hst = (uint8_t*)pinned(c, "clahe_io", nin);
    uint8_t* dimg = (uint8_t*)scratch(c, "clahe_img", nin);
    double* dmean = hist_mean ? (double*)scratch(c, "clahe_mean", sizeof(double)) : nullptr;
    if (!hst || !dimg || (hist_mean && !dmean)) return set_err(c, GVX_ERR_OOM, "CLAHE staging");
    hipStreamSynchronize(c->stream);  // staging buffer reuse
    for (int y = 0; y < h; ++y) std::memcpy(hst + (size_t)y * w * ch, src + (size_t)y * src_stride, (size_t)w * ch);
    hipError_t e = hipMemcpyAsync(dimg, hst, nin, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "hipMemcpyAsync(CLAHE in)");
    s = clahe_enqueue(c, 1, w, h, dimg, (int64_t)nin, w * ch, dimg, (int64_t)nb, w, cp, dmean);
    if (s) return s;
    e = hipMemcpyAsync(hst, dimg, nb, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && hist_mean) e = hipMemcpyAsync(hist_mean, dmean, sizeof(double), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "CLAHE copy-out");
    for (int y = 0; y < h; ++y) std::memcpy(dst + (size_t)y * dst_stride, hst + (size_t)y * w, w);
    return GVX_OK;
}

// CLAHE straight into the frame's padded level-0 slot, ring included (frames of
// at least 66 x 66 px: the ring is then a single-bounce REFLECT_101 copy), then
// levels >= 1 from that slot: no level-0 copy pass.  src_index: the frame is
// d_gray + (*src_index) * img_stride, picked on the device.
static gvx_status preprocess_into_slot(gvx_ctx* c, uint64_t id, const uint8_t* d_gray, int64_t img_stride,
                                       const int32_t* src_index, int32_t n_src, int32_t w, int32_t h, int32_t stride,
                                       const gvx_clahe_params* cp, const gvx_klt_params* p, double* d_hist_mean) {
    Frame* f = nullptr;
    gvx_status s = frame_slot(c, id, w, h, p, &f);
    if (s) return s;
    const PyrLayout& lay = f->lay;
    uint8_t* slot0 = f->pyr + lay.off[0] + (int64_t)PAD * lay.pitch[0] + PAD;
    s = clahe_enqueue(c, 1, w, h, d_gray, img_stride, stride, slot0, lay.bytes, lay.pitch[0], cp, d_hist_mean,
                      src_index, n_src, 1);
    if (s) return s;
    hipError_t e = launch_build_pyramids(c, slot0, lay.bytes, lay.pitch[0], 1, lay, f->pyr, false, nullptr, 0, true);
    return hip_err(c, e, "pyramid kernels");
}
static bool ring_in_apply(int w, int h) { return w >= 2 * PAD + 2 && h >= 2 * PAD + 2; }

gvx_status gvx_frame_preprocess_indexed_dev(gvx_ctx* c, uint64_t id, const uint8_t* d_frames,
                                            int64_t frame_stride, const int32_t* d_index, int32_t n_frames,
                                            int32_t w, int32_t h,
                                            int32_t stride, const gvx_clahe_params* cp, const gvx_klt_params* p,
                                            double* d_hist_mean) {
    if (!c) return GVX_ERR_INVALID;
    if (!d_frames || !d_index || n_frames <= 0 || w <= 0 || h <= 0 || stride < chan_of(cp) * w ||
        frame_stride < (int64_t)stride * (h - 1) + chan_of(cp) * w)
        return set_err(c, GVX_ERR_INVALID, "bad frame sequence");
    if (!ring_in_apply(w, h)) return set_err(c, GVX_ERR_INVALID, "indexed preprocessing needs frames >= 66 x 66");
    gvx_status s = check_clahe(c, w, h, cp);
    if (s) return s;
    hipSetDevice(c->device);
    return preprocess_into_slot(c, id, d_frames, frame_stride, d_index, n_frames, w, h, stride, cp, p, d_hist_mean);
}

gvx_status gvx_frame_preprocess_dev(gvx_ctx* c, uint64_t id, const uint8_t* d_gray, int32_t w, int32_t h,
                                    int32_t stride, const gvx_clahe_params* cp, const gvx_klt_params* p,
                                    double* d_hist_mean, uint8_t* d_clahe_out) {
    if (!c) return GVX_ERR_INVALID;
    if (!d_gray || w <= 0 || h <= 0 || stride < chan_of(cp) * w) return set_err(c, GVX_ERR_INVALID, "bad frame");
    gvx_status s = check_clahe(c, w, h, cp);
    if (s) return s;
    hipSetDevice(c->device);
    if (!d_clahe_out && ring_in_apply(w, h))
        return preprocess_into_slot(c, id, d_gray, (int64_t)h * stride, nullptr, 0, w, h, stride, cp, p,
                                    d_hist_mean);
    const size_t nb = (size_t)w * h;
    uint8_t* eq = d_clahe_out ? d_clahe_out : (uint8_t*)scratch(c, "preproc_eq", nb);
    if (!eq) return set_err(c, GVX_ERR_OOM, "preprocess scratch");
    s = clahe_enqueue(c, 1, w, h, d_gray, (int64_t)h * stride, stride, eq, (int64_t)nb, w, cp, d_hist_mean);
    if (s) return s;
    // the pyramid build copies the equalised level 0 into the frame's padded slot
    // (stream order: the scratch is not reused before that copy ran)
    return gvx_frame_put_dev(c, id, eq, w, h, w, p);
}

gvx_status gvx_frame_preprocess(gvx_ctx* c, uint64_t id, const uint8_t* gray, int32_t w, int32_t h,
                                int32_t stride, const gvx_clahe_params* cp, const gvx_klt_params* p,
                                double* hist_mean, uint8_t* clahe_out) {
    if (!c) return GVX_ERR_INVALID;
    const int ch = chan_of(cp);
    if (!gray || w <= 0 || h <= 0 || stride < ch * w) return set_err(c, GVX_ERR_INVALID, "bad frame");
    gvx_status s = check_clahe(c, w, h, cp);
    if (s) return s;
    hipSetDevice(c->device);
    const size_t nb = (size_t)w * h, nin = nb * ch;
    uint8_t* hst = (uint8_t*)pinned(c, "preproc_io", nin);
    uint8_t* din = (uint8_t*)scratch(c, "preproc_in", nin);
    uint8_t* dout = (uint8_t*)scratch(c, "preproc_out", nb);
    double* dmean = hist_mean ? (double*)scratch(c, "preproc_mean", sizeof(double)) : nullptr;
    if (!hst || !din || !dout || (hist_mean && !dmean)) return set_err(c, GVX_ERR_OOM, "preprocess staging");
    hipStreamSynchronize(c->stream);  // staging buffer reuse
    for (int y = 0; y < h; ++y) std::memcpy(hst + (size_t)y * w * ch, gray + (size_t)y * stride, (size_t)w * ch);
    hipError_t e = hipMemcpyAsync(din, hst, nin, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "hipMemcpyAsync(frame)");
    s = gvx_frame_preprocess_dev(c, id, din, w, h, w * ch, cp, p, dmean, dout);
    if (s) return s;
    if (clahe_out) e = hipMemcpyAsync(hst, dout, nb, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && hist_mean)
        e = hipMemcpyAsync(hist_mean, dmean, sizeof(double), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "preprocess copy-out");
    if (clahe_out) std::memcpy(clahe_out, hst, nb);
    return GVX_OK;
}
