// api.cpp -- C ABI entry points of libgvx (include/gvx.h): context, frame cache,
// KLT dispatch, profiling.  Compiled with hipcc for gfx950 (host code only here).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstring>

#include "gvx_internal.h"

using namespace gvx;

namespace gvx {

gvx_status set_err(gvx_ctx* c, gvx_status s, const char* fmt, ...) {
    if (c) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        c->err = buf;
    }
    return s;
}

gvx_status hip_err(gvx_ctx* c, hipError_t e, const char* what) {
    if (e == hipSuccess) return GVX_OK;
    return set_err(c, e == hipErrorOutOfMemory ? GVX_ERR_OOM : GVX_ERR_HIP, "%s: %s", what,
                   hipGetErrorString(e));
}

// both streams of the context (the side branch's too) before memory is freed
void sync_all(gvx_ctx* c) {
    hipStreamSynchronize(c->main);
    if (c->side) hipStreamSynchronize(c->side);
}

void* scratch(gvx_ctx* c, const std::string& name, size_t bytes) {
    DevBuf& b = c->dev[name];
    if (b.bytes >= bytes && b.p) return b.p;
    if (c->capturing) {  // growing would synchronise the captured stream
        c->capture_failed = true;
        return nullptr;
    }
    ++c->mem_gen;
    if (b.p) {
        sync_all(c);
        hipFree(b.p);
        b.p = nullptr;
        b.bytes = 0;
    }
    size_t want = bytes < 256 ? 256 : bytes;
    if (hipMalloc(&b.p, want) != hipSuccess) {
        b.p = nullptr;
        return nullptr;
    }
    b.bytes = want;
    b.fresh = true;
    return b.p;
}

void* pinned(gvx_ctx* c, const std::string& name, size_t bytes) {
    DevBuf& b = c->pinned[name];
    if (b.bytes >= bytes && b.p) return b.p;
    if (c->capturing) {
        c->capture_failed = true;
        return nullptr;
    }
    ++c->mem_gen;
    if (b.p) {
        sync_all(c);
        hipHostFree(b.p);
        b.p = nullptr;
        b.bytes = 0;
    }
    size_t want = bytes < 256 ? 256 : bytes;
    if (hipHostMalloc(&b.p, want, hipHostMallocDefault) != hipSuccess) {
        b.p = nullptr;
        return nullptr;
    }
    b.bytes = want;
    return b.p;
}

static hipEvent_t get_event(gvx_ctx* c) {
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
}

void prof_begin(gvx_ctx* c, const char* fam, hipEvent_t* a) {
    (void)fam;
    if (!c->prof) return;
    *a = get_event(c);
    hipEventRecord(*a, c->stream);
}

void prof_end(gvx_ctx* c, const char* fam, hipEvent_t a) {
    if (!c->prof) return;
    hipEvent_t b = get_event(c);
    hipEventRecord(b, c->stream);
    prof_push(c, fam, a, b);
}

hipEvent_t prof_event(gvx_ctx* c) { return get_event(c); }

void prof_push(gvx_ctx* c, const char* fam, hipEvent_t a, hipEvent_t b) {
    c->pending.push_back({fam, a, b});
    if (c->pending.size() > 4096) prof_drain(c);
}

void prof_drain(gvx_ctx* c) {
    if (c->pending.empty()) return;
    // events may sit on the context stream and on its branch stream
    hipStreamSynchronize(c->main);
    if (c->side) hipStreamSynchronize(c->side);
    for (auto& p : c->pending) {
        float ms = 0;
        hipEventElapsedTime(&ms, p.a, p.b);
        auto& e = c->prof_acc[p.fam];
        e.ms += ms;
        e.launches += 1;
        c->event_pool.push_back(p.a);
        c->event_pool.push_back(p.b);
    }
    c->pending.clear();
}

}  // namespace gvx

extern "C" {

const char* gvx_version(void) { return "gvx 0.1 gfx950"; }

const char* gvx_status_string(gvx_status s) {
    switch (s) {
        case GVX_OK: return "ok";
        case GVX_ERR_INVALID: return "invalid argument";
        case GVX_ERR_NO_DEVICE: return "no device";
        case GVX_ERR_HIP: return "hip error";
        case GVX_ERR_OOM: return "out of memory";
        case GVX_ERR_NOT_FOUND: return "not found";
        case GVX_ERR_UNSUPPORTED: return "unsupported";
        case GVX_ERR_NUMERIC: return "not positive definite";
        default: return "unknown";
    }
}

gvx_status gvx_create(int32_t device, gvx_ctx** out) {
    if (!out) return GVX_ERR_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return GVX_ERR_NO_DEVICE;
    if (device < 0 || device >= n) return GVX_ERR_INVALID;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return GVX_ERR_NO_DEVICE;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return GVX_ERR_NO_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return GVX_ERR_HIP;
    gvx_ctx* c = new gvx_ctx();
    c->device = device;
    c->n_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    {
        const char* sp = std::getenv("GVX_SIDE_LOW_PRIO");
        c->side_low_prio = sp ? std::atoi(sp) : 0;
    }
    hipError_t se;
    if (c->side_low_prio) {
        int least = 0, greatest = 0;
        se = hipDeviceGetStreamPriorityRange(&least, &greatest);
        if (se == hipSuccess)
            se = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, c->side_low_prio == 2 ? least : greatest);
    } else {
        se = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    }
    if (se != hipSuccess) {
        delete c;
        return GVX_ERR_HIP;
    }
    c->main = c->stream;
    {
        // A/B switches are read once, here (not per launch)
        const char* e = std::getenv("GVX_PREINT_ONEPHASE");
        if (e && std::atoi(e) != 0) c->preint_path = GVX_PREINT_PATH_ONEPHASE;
        const char* f = std::getenv("GVX_FACTORSET_D2H");
        c->factorset_d2h = f && std::atoi(f) != 0;
        // GVX_PROF_MARKERS=1: profiled launches bracketed by recorded events
        // instead of events attached to the dispatch (the r05_m1 queue-abort A/B)
        const char* m = std::getenv("GVX_PROF_MARKERS");
        c->prof_markers = m && std::atoi(m) != 0;
        const char* k = std::getenv("GVX_KLT_LPP");
        if (k) c->klt_lpp = std::max(0, std::atoi(k));
        const char* sk = std::getenv("GVX_KLT_SUPER");
        if (sk) c->klt_super = std::max(8, std::atoi(sk));
        const char* pw = std::getenv("GVX_PYR_WPB");
        if (pw) c->pyr_wpb = std::atoi(pw) == 4 ? 4 : 1;
        const char* po = std::getenv("GVX_PYR_ORDER");
        if (po) c->pyr_order = std::atoi(po) != 0;
        const char* fc = std::getenv("GVX_FUSED_COMPACT");
        if (fc) c->fused_compact = std::atoi(fc) != 0;
    }
    *out = c;
    return GVX_OK;
}

void gvx_destroy(gvx_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->main);
    if (c->side) hipStreamSynchronize(c->side);
    for (auto& f : c->frames) {
        hipFree(f.second.pyr);
        hipFree(f.second.eig);
    }
    for (auto& b : c->dev) hipFree(b.second.p);
    for (auto& b : c->pinned) hipHostFree(b.second.p);
    for (auto& p : c->pending) {
        hipEventDestroy(p.a);
        hipEventDestroy(p.b);
    }
    for (auto e : c->event_pool) hipEventDestroy(e);
    if (c->side) {
        hipStreamSynchronize(c->side);
        hipStreamDestroy(c->side);
    }
    if (c->fork_ev) hipEventDestroy(c->fork_ev);
    if (c->join_ev) hipEventDestroy(c->join_ev);
    hipStreamDestroy(c->main);
    delete c;
}

const char* gvx_last_error(const gvx_ctx* c) { return c ? c->err.c_str() : ""; }

gvx_status gvx_sync(gvx_ctx* c) {
    if (!c) return GVX_ERR_INVALID;
    if (c->side) {
        const hipError_t e = hipStreamSynchronize(c->side);
        if (e != hipSuccess) return hip_err(c, e, "hipStreamSynchronize");
        if (!c->in_branch) c->branch_open = false;  // the branch's work is done: nothing left to join
    }
    return hip_err(c, hipStreamSynchronize(c->main), "hipStreamSynchronize");
}

void* gvx_get_stream(gvx_ctx* c) { return c ? (void*)c->stream : nullptr; }

gvx_status gvx_set_klt_phases(gvx_ctx* c, int32_t levels_per_phase, int32_t groups_per_chunk) {
    if (!c) return GVX_ERR_INVALID;
    if (levels_per_phase < 0 || levels_per_phase > gvx::MAX_LEVELS)
        return set_err(c, GVX_ERR_INVALID, "levels per phase %d (0..%d)", levels_per_phase, gvx::MAX_LEVELS);
    if (groups_per_chunk < 0 || (groups_per_chunk > 0 && groups_per_chunk < 8))
        return set_err(c, GVX_ERR_INVALID, "groups per chunk %d (0 or >= 8)", groups_per_chunk);
    c->klt_lpp = levels_per_phase;
    if (groups_per_chunk) c->klt_super = groups_per_chunk;
    return GVX_OK;
}

gvx_status gvx_profile_enable(gvx_ctx* c, int32_t on) {
    if (!c) return GVX_ERR_INVALID;
    if (!on) prof_drain(c);
    c->prof = on != 0;
    return GVX_OK;
}

gvx_status gvx_profile_read(gvx_ctx* c, const char* fam, double* ms, int64_t* launches) {
    if (!c || !fam) return GVX_ERR_INVALID;
    prof_drain(c);
    auto it = c->prof_acc.find(fam);
    if (ms) *ms = it == c->prof_acc.end() ? 0.0 : it->second.ms;
    if (launches) *launches = it == c->prof_acc.end() ? 0 : it->second.launches;
    return GVX_OK;
}

gvx_status gvx_profile_reset(gvx_ctx* c) {
    if (!c) return GVX_ERR_INVALID;
    prof_drain(c);
    c->prof_acc.clear();
    return GVX_OK;
}

void gvx_klt_params_default(gvx_klt_params* p) {
    if (!p) return;
    p->win = 21;
    p->max_level = 3;
    p->max_iter = 30;
    p->eps = 0.01;
    p->use_initial_flow = 1;
    p->min_eig = 1e-4f;
    p->accum = GVX_LK_ACCUM_EXACT;
}

static gvx_status check_klt_params(gvx_ctx* c, const gvx_klt_params* p) {
    if (!p) return set_err(c, GVX_ERR_INVALID, "null klt params");
    if (p->accum < GVX_LK_ACCUM_EXACT || p->accum > GVX_LK_ACCUM_F32_SIMD4)
        return set_err(c, GVX_ERR_INVALID, "unknown LK accumulation order %d", p->accum);
    if (p->win != WIN)
        return set_err(c, GVX_ERR_UNSUPPORTED, "device LK supports win=21 only (got %d)", p->win);
    if (p->max_level < 0 || p->max_level >= MAX_LEVELS)
        return set_err(c, GVX_ERR_INVALID, "max_level %d out of range", p->max_level);
    return GVX_OK;
}

static KltArgs klt_args(const gvx_klt_params* p) {
    KltArgs a{};
    // calcOpticalFlowPyrLK criteria normalisation (COUNT and EPS both set)
    int it = p->max_iter;
    a.max_iter = it < 0 ? 0 : (it > 100 ? 100 : it);
    double e = p->eps < 0 ? 0.0 : (p->eps > 10.0 ? 10.0 : p->eps);
    a.crit_eps = e * e;
    a.min_eig = p->min_eig;
    a.use_initial_flow = p->use_initial_flow;
    a.accum = p->accum;
    return a;
}

gvx_status gvx_frame_put(gvx_ctx* c, uint64_t id, const uint8_t* gray, int32_t w, int32_t h,
                         int32_t stride, const gvx_klt_params* p) {
    if (!c || !gray || w <= 0 || h <= 0 || stride < w) return set_err(c, GVX_ERR_INVALID, "bad frame");
    gvx_status s = check_klt_params(c, p);
    if (s) return s;
    if (w <= WIN || h <= WIN) return set_err(c, GVX_ERR_INVALID, "frame smaller than the window");
    hipSetDevice(c->device);
    PyrLayout lay = make_layout(w, h, p->max_level, p->win);
    Frame& f = c->frames[id];
    if (!f.pyr || f.lay.bytes < lay.bytes) {
        if (c->capturing) {
            if (!f.pyr) c->frames.erase(id);
            c->capture_failed = true;
            return set_err(c, GVX_ERR_INVALID, "frame %llu needs a (re)allocation during a graph capture",
                           (unsigned long long)id);
        }
        ++c->mem_gen;
        if (f.pyr) {
            sync_all(c);
            hipFree(f.pyr);
            f.pyr = nullptr;
        }
        hipError_t e = hipMalloc(&f.pyr, lay.bytes);
        if (e != hipSuccess) {
            c->frames.erase(id);
            return hip_err(c, e, "hipMalloc(pyramid)");
        }
    }
    f.lay = lay;
    f.w = w;
    f.h = h;
    ++f.gen;
    size_t nb = (size_t)h * w;
    uint8_t* hst = (uint8_t*)pinned(c, "frame_in", nb);
    uint8_t* dsrc = (uint8_t*)scratch(c, "frame_in", nb);
    if (!hst || !dsrc) return set_err(c, GVX_ERR_OOM, "frame staging");
    hipStreamSynchronize(c->stream);  // staging buffer reuse
    for (int y = 0; y < h; ++y) std::memcpy(hst + (size_t)y * w, gray + (size_t)y * stride, w);
    hipError_t e = hipMemcpyAsync(dsrc, hst, nb, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "hipMemcpyAsync(frame)");
    e = launch_build_pyramids(c, dsrc, (int64_t)nb, w, 1, lay, f.pyr, true);
    if (e != hipSuccess) return hip_err(c, e, "pyramid kernels");
    return hip_err(c, hipStreamSynchronize(c->stream), "frame_put sync");
}

gvx_status gvx_frame_put_dev(gvx_ctx* c, uint64_t id, const uint8_t* d_gray, int32_t w, int32_t h,
                             int32_t stride, const gvx_klt_params* p) {
    if (!c || !d_gray || w <= 0 || h <= 0 || stride < w) return set_err(c, GVX_ERR_INVALID, "bad frame");
    Frame* fp = nullptr;
    gvx_status s = frame_slot(c, id, w, h, p, &fp);
    if (s) return s;
    Frame& f = *fp;
    const PyrLayout& lay = f.lay;
    // the padded level-0 copy reads the caller's device image in place (any stride)
    hipError_t e = launch_build_pyramids(c, d_gray, (int64_t)h * stride, stride, 1, lay, f.pyr, true);
    return hip_err(c, e, "pyramid kernels");
}

gvx_status gvx_frame_drop(gvx_ctx* c, uint64_t id) {
    if (!c) return GVX_ERR_INVALID;
    auto it = c->frames.find(id);
    if (it == c->frames.end()) return set_err(c, GVX_ERR_NOT_FOUND, "frame %llu", (unsigned long long)id);
    if (c->capturing) return set_err(c, GVX_ERR_INVALID, "gvx_frame_drop during a graph capture");
    ++c->mem_gen;
    sync_all(c);
    hipFree(it->second.pyr);
    hipFree(it->second.eig);
    c->frames.erase(it);
    return GVX_OK;
}

gvx_status gvx_frame_level(gvx_ctx* c, uint64_t id, int32_t level, uint8_t* out, int32_t* w, int32_t* h) {
    if (!c) return GVX_ERR_INVALID;
    auto it = c->frames.find(id);
    if (it == c->frames.end()) return set_err(c, GVX_ERR_NOT_FOUND, "frame %llu", (unsigned long long)id);
    const PyrLayout& L = it->second.lay;
    if (level < 0 || level >= L.nlev) return set_err(c, GVX_ERR_INVALID, "level %d", level);
    if (w) *w = L.w[level];
    if (h) *h = L.h[level];
    if (!out) return GVX_OK;
    const uint8_t* src = it->second.pyr + L.off[level] + (int64_t)PAD * L.pitch[level] + PAD;
    hipError_t e = hipMemcpy2DAsync(out, L.w[level], src, L.pitch[level], L.w[level], L.h[level],
                                    hipMemcpyDeviceToHost, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "copy level");
    return hip_err(c, hipStreamSynchronize(c->stream), "copy level sync");
}

gvx_status gvx_frame_level_padded(gvx_ctx* c, uint64_t id, int32_t level, int32_t pad, uint8_t* out) {
    static_assert(GVX_PYR_PAD == PAD, "ABI pad constant");
    if (!c) return GVX_ERR_INVALID;
    auto it = c->frames.find(id);
    if (it == c->frames.end()) return set_err(c, GVX_ERR_NOT_FOUND, "frame %llu", (unsigned long long)id);
    const PyrLayout& L = it->second.lay;
    if (level < 0 || level >= L.nlev) return set_err(c, GVX_ERR_INVALID, "level %d", level);
    if (pad < 0 || pad > PAD || !out) return set_err(c, GVX_ERR_INVALID, "pad %d", pad);
    const uint8_t* src = it->second.pyr + L.off[level] + (int64_t)(PAD - pad) * L.pitch[level] + (PAD - pad);
    const int w = L.w[level] + 2 * pad, h = L.h[level] + 2 * pad;
    hipError_t e = hipMemcpy2DAsync(out, w, src, L.pitch[level], w, h, hipMemcpyDeviceToHost, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "copy level");
    return hip_err(c, hipStreamSynchronize(c->stream), "copy level sync");
}

gvx_status gvx_pyramid_layout(int32_t w, int32_t h, int32_t max_level, int32_t* nlev, int64_t* off,
                              int32_t* pitch, int32_t* lw, int32_t* lh, int64_t* bytes) {
    if (w <= WIN || h <= WIN || max_level < 0) return GVX_ERR_INVALID;
    const PyrLayout L = make_layout(w, h, max_level, WIN);
    if (nlev) *nlev = L.nlev;
    for (int l = 0; l < L.nlev; ++l) {
        if (off) off[l] = L.off[l];
        if (pitch) pitch[l] = L.pitch[l];
        if (lw) lw[l] = L.w[l];
        if (lh) lh[l] = L.h[l];
    }
    if (bytes) *bytes = L.bytes;
    return GVX_OK;
}

gvx_status gvx_build_pyramids_dev(gvx_ctx* c, int32_t n_img, int32_t w, int32_t h, const uint8_t* d_imgs,
                                  int64_t img_stride, int32_t stride, int32_t max_level, uint8_t* d_out) {
    if (!c) return GVX_ERR_INVALID;
    if (n_img < 0 || w <= WIN || h <= WIN || stride < w || img_stride < (int64_t)stride * (h - 1) + w ||
        max_level < 0 || max_level >= MAX_LEVELS)
        return set_err(c, GVX_ERR_INVALID, "bad pyramid batch");
    if (n_img == 0) return GVX_OK;
    if (!d_imgs || !d_out) return set_err(c, GVX_ERR_INVALID, "bad pyramid batch pointers");
    hipSetDevice(c->device);
    const PyrLayout lay = make_layout(w, h, max_level, WIN);
    hipError_t e = launch_build_pyramids(c, d_imgs, img_stride, stride, n_img, lay, d_out, false);
    return hip_err(c, e, "pyramid kernels");
}

// Shared single-pair path of gvx_klt / gvx_klt_fb.
static gvx_status klt_single(gvx_ctx* c, uint64_t prev_id, uint64_t next_id, const float* prev_xy,
                             float* next_xy, float* back_xy, uint8_t* flags_out, float* err,
                             int32_t n, const gvx_klt_params* p, int mode, double fb, double border,
                             int cam_w, int cam_h, int32_t* kept_idx, int32_t* n_kept) {
    auto ip = c->frames.find(prev_id), in = c->frames.find(next_id);
    if (ip == c->frames.end() || in == c->frames.end())
        return set_err(c, GVX_ERR_NOT_FOUND, "frame not cached");
    const Frame& fp = ip->second;
    const Frame& fn = in->second;
    if (fp.w != fn.w || fp.h != fn.h) return set_err(c, GVX_ERR_INVALID, "frame sizes differ");
    PyrLayout lay = make_layout(fp.w, fp.h, p->max_level, p->win);
    if (lay.nlev > fp.lay.nlev || lay.nlev > fn.lay.nlev)
        return set_err(c, GVX_ERR_INVALID, "frames were put with a smaller max_level");
    // the cached layouts may have more levels; offsets of the first nlev levels agree
    lay = fp.lay;
    lay.nlev = make_layout(fp.w, fp.h, p->max_level, p->win).nlev;
    hipSetDevice(c->device);
    // staging: pts in (prev, next) | out (next, back, flags, err, kept, n_kept)
    size_t fb_bytes = sizeof(float) * 2 * (size_t)n;
    size_t need = 4 * fb_bytes + (size_t)n + sizeof(float) * n + sizeof(int32_t) * (n + 1) + 256;
    char* h = (char*)pinned(c, "klt", need);
    char* d = (char*)scratch(c, "klt", need);
    if (!h || !d) return set_err(c, GVX_ERR_OOM, "klt staging");
    // no wait here: the staging buffers are only in flight inside this call (it
    // ends with a synchronisation), so the points are staged and the upload and
    // launch queue up behind the frames' preprocessing already on the stream
    float* h_prev = (float*)h;
    float* h_next = (float*)(h + fb_bytes);
    float* h_back = (float*)(h + 2 * fb_bytes);
    float* h_err = (float*)(h + 3 * fb_bytes);
    int32_t* h_kept = (int32_t*)(h + 3 * fb_bytes + sizeof(float) * n);
    int32_t* h_nkept = h_kept + n;
    uint8_t* h_flags = (uint8_t*)(h_nkept + 1);
    float* d_prev = (float*)d;
    float* d_next = (float*)(d + fb_bytes);
    float* d_back = (float*)(d + 2 * fb_bytes);
    float* d_err = (float*)(d + 3 * fb_bytes);
    int32_t* d_kept = (int32_t*)(d + 3 * fb_bytes + sizeof(float) * n);
    int32_t* d_nkept = d_kept + n;
    uint8_t* d_flags = (uint8_t*)(d_nkept + 1);
    std::memcpy(h_prev, prev_xy, fb_bytes);
    if (p->use_initial_flow)
        std::memcpy(h_next, next_xy, fb_bytes);
    else
        std::memcpy(h_next, prev_xy, fb_bytes);
    hipError_t e = hipMemcpyAsync(d_prev, h_prev, 2 * fb_bytes, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "H2D points");
    KltArgs a = klt_args(p);
    a.n_pairs = 1;
    a.n_pts = n;
    a.mode = mode;
    a.fb_thresh = fb;
    a.border = border;
    a.cam_w = cam_w;
    a.cam_h = cam_h;
    const Level0 l0{fp.pyr + lay.off[0], fn.pyr + lay.off[0], 0, 0, PAD * lay.pitch[0] + PAD, lay.pitch[0], 0};
    if (mode == 1)
        e = launch_klt_compact(c, a, lay, fp.pyr, fn.pyr, 0, 0, l0, d_prev, d_next, d_back, d_flags, d_err, d_kept,
                               d_nkept);
    else
        e = launch_klt(c, a, lay, fp.pyr, fn.pyr, 0, 0, l0, d_prev, d_next, nullptr, d_flags, d_err);
    if (e != hipSuccess) return hip_err(c, e, "klt kernels");
    // one D2H of next | back | err | kept | n_kept | flags
    const size_t tail = 2 * fb_bytes + sizeof(float) * n + sizeof(int32_t) * (n + 1) + n;
    e = hipMemcpyAsync(h_next, d_next, tail, hipMemcpyDeviceToHost, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "D2H results");
    e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "klt sync");
    std::memcpy(next_xy, h_next, fb_bytes);
    if (mode == 0) {
        if (flags_out)
            for (int i = 0; i < n; ++i) flags_out[i] = h_flags[i] & 1;
        if (err) std::memcpy(err, h_err, sizeof(float) * n);
        return GVX_OK;
    }
    if (back_xy) std::memcpy(back_xy, h_back, fb_bytes);
    if (flags_out) std::memcpy(flags_out, h_flags, n);
    if (kept_idx) std::memcpy(kept_idx, h_kept, sizeof(int32_t) * (*h_nkept));
    if (n_kept) *n_kept = *h_nkept;
    return GVX_OK;
}

gvx_status gvx_klt(gvx_ctx* c, uint64_t prev_id, uint64_t next_id, const float* prev_xy,
                   float* next_xy, uint8_t* status, float* err, int32_t n, const gvx_klt_params* p) {
    if (!c) return GVX_ERR_INVALID;
    gvx_status s = check_klt_params(c, p);
    if (s) return s;
    if (n < 0 || (n > 0 && (!prev_xy || !next_xy))) return set_err(c, GVX_ERR_INVALID, "bad points");
    if (n == 0) return GVX_OK;
    return klt_single(c, prev_id, next_id, prev_xy, next_xy, nullptr, status, err, n, p, 0, 0, 0, 0,
                      0, nullptr, nullptr);
}

gvx_status gvx_klt_fb(gvx_ctx* c, uint64_t prev_id, uint64_t next_id, const float* prev_xy,
                      float* next_xy, float* back_xy, uint8_t* status_fwd, uint8_t* status_bwd,
                      uint8_t* keep, int32_t* kept_idx, int32_t* n_kept, int32_t n,
                      double fb_thresh, double border, int32_t cam_w, int32_t cam_h,
                      const gvx_klt_params* p) {
    if (!c) return GVX_ERR_INVALID;
    gvx_status s = check_klt_params(c, p);
    if (s) return s;
    if (n < 0 || (n > 0 && (!prev_xy || !next_xy)) || !n_kept)
        return set_err(c, GVX_ERR_INVALID, "bad points");
    if (n == 0) {
        *n_kept = 0;
        return GVX_OK;
    }
    std::vector<uint8_t> flags(n);
    s = klt_single(c, prev_id, next_id, prev_xy, next_xy, back_xy, flags.data(), nullptr, n, p, 1,
                   fb_thresh, border, cam_w, cam_h, kept_idx, n_kept);
    if (s) return s;
    for (int i = 0; i < n; ++i) {
        if (status_fwd) status_fwd[i] = flags[i] & 1;
        if (status_bwd) status_bwd[i] = (flags[i] >> 1) & 1;
        if (keep) keep[i] = (flags[i] >> 2) & 1;
    }
    return GVX_OK;
}

// LK / FB + compaction of a batch over built pyramids (levels >= 1 at pyr_prev /
// pyr_next + i * lay.bytes; level 0 read in place from the caller's images).
static gvx_status klt_batch_on_pyramids(gvx_ctx* c, const PyrLayout& lay, int32_t n_pairs, int32_t w, int32_t h,
                                        const uint8_t* d_prev, const uint8_t* d_next, const uint8_t* pyr_prev,
                                        const uint8_t* pyr_next, int32_t n_pts, const float* d_prev_xy,
                                        const float* d_init_xy, float* d_next_xy, float* d_back_xy, uint8_t* d_flags,
                                        int32_t* d_kept_idx, int32_t* d_n_kept, double fb_thresh, double border,
                                        int32_t cam_w, int32_t cam_h, const gvx_klt_params* p) {
    hipError_t e;
    if (n_pts == 0) {
        e = hipMemsetAsync(d_n_kept, 0, sizeof(int32_t) * n_pairs, c->stream);
        return hip_err(c, e, "memset n_kept");
    }
    KltArgs a = klt_args(p);
    a.n_pairs = n_pairs;
    a.n_pts = n_pts;
    a.mode = 1;
    a.fb_thresh = fb_thresh;
    a.border = border;
    a.cam_w = cam_w;
    a.cam_h = cam_h;
    // without OPTFLOW_USE_INITIAL_FLOW the kernel starts from prevPts and never
    // reads the initial flow
    a.init_xy = d_init_xy;
    const Level0 l0{d_prev, d_next, (int64_t)w * h, (int64_t)w * h, 0, w, 1};
    e = launch_klt_compact(c, a, lay, pyr_prev, pyr_next, lay.bytes, lay.bytes, l0, d_prev_xy, d_next_xy,
                           d_back_xy, d_flags, nullptr, d_kept_idx, d_n_kept);
    return hip_err(c, e, "klt kernels");
}

static gvx_status check_batch(gvx_ctx* c, int32_t n_pairs, int32_t w, int32_t h, const uint8_t* d_prev,
                              const uint8_t* d_next, int32_t n_pts, const float* d_prev_xy, float* d_next_xy,
                              uint8_t* d_flags, int32_t* d_kept_idx, int32_t* d_n_kept) {
    if (n_pairs < 0 || n_pts < 0 || w <= WIN || h <= WIN || !d_prev || !d_next)
        return set_err(c, GVX_ERR_INVALID, "bad batch");
    if (n_pts > 0 && (!d_prev_xy || !d_next_xy || !d_flags || !d_kept_idx || !d_n_kept))
        return set_err(c, GVX_ERR_INVALID, "bad batch pointers");
    return GVX_OK;
}

gvx_status gvx_klt_fb_batch_init_dev(gvx_ctx* c, int32_t n_pairs, int32_t w, int32_t h,
                                     const uint8_t* d_prev, const uint8_t* d_next, int32_t n_pts,
                                     const float* d_prev_xy, const float* d_init_xy, float* d_next_xy,
                                     float* d_back_xy, uint8_t* d_flags, int32_t* d_kept_idx, int32_t* d_n_kept,
                                     double fb_thresh, double border, int32_t cam_w, int32_t cam_h,
                                     const gvx_klt_params* p) {
    if (!c) return GVX_ERR_INVALID;
    gvx_status s = check_klt_params(c, p);
    if (s) return s;
    s = check_batch(c, n_pairs, w, h, d_prev, d_next, n_pts, d_prev_xy, d_next_xy, d_flags, d_kept_idx, d_n_kept);
    if (s) return s;
    if (n_pairs == 0) return GVX_OK;
    hipSetDevice(c->device);
    PyrLayout lay = make_layout(w, h, p->max_level, p->win);
    uint8_t* pyr = (uint8_t*)scratch(c, "batch_pyr", (size_t)lay.bytes * 2 * n_pairs);
    if (!pyr) return set_err(c, GVX_ERR_OOM, "batch pyramids (%lld bytes)", (long long)lay.bytes * 2 * n_pairs);
    uint8_t* pyr_prev = pyr;
    uint8_t* pyr_next = pyr + (size_t)lay.bytes * n_pairs;
    // level 0 stays in the caller's images; levels >= 1 go to the pyramid slots
    // one launch for both frames of every pair (pyr_next follows pyr_prev)
    hipError_t e = launch_build_pyramids(c, d_prev, (int64_t)w * h, w, 2 * n_pairs, lay, pyr_prev, false, d_next,
                                         n_pairs);
    if (e != hipSuccess) return hip_err(c, e, "pyramid kernels");
    return klt_batch_on_pyramids(c, lay, n_pairs, w, h, d_prev, d_next, pyr_prev, pyr_next, n_pts, d_prev_xy,
                                 d_init_xy, d_next_xy, d_back_xy, d_flags, d_kept_idx, d_n_kept, fb_thresh, border,
                                 cam_w, cam_h, p);
}

gvx_status gvx_klt_batch_pyramids_dev(gvx_ctx* c, int32_t n_pairs, int32_t w, int32_t h, const uint8_t* d_prev,
                                      const uint8_t* d_next, int32_t max_level, uint8_t* d_pyr) {
    if (!c) return GVX_ERR_INVALID;
    if (n_pairs < 0 || w <= WIN || h <= WIN || max_level < 0 || max_level >= MAX_LEVELS)
        return set_err(c, GVX_ERR_INVALID, "bad pyramid batch");
    if (n_pairs == 0) return GVX_OK;
    if (!d_prev || !d_next || !d_pyr) return set_err(c, GVX_ERR_INVALID, "bad pyramid batch pointers");
    hipSetDevice(c->device);
    const PyrLayout lay = make_layout(w, h, max_level, WIN);
    hipError_t e = launch_build_pyramids(c, d_prev, (int64_t)w * h, w, 2 * n_pairs, lay, d_pyr, false, d_next,
                                         n_pairs);
    return hip_err(c, e, "pyramid kernels");
}

gvx_status gvx_klt_fb_batch_pyr_dev(gvx_ctx* c, int32_t n_pairs, int32_t w, int32_t h, const uint8_t* d_prev,
                                    const uint8_t* d_next, const uint8_t* d_pyr, int32_t n_pts,
                                    const float* d_prev_xy, const float* d_init_xy, float* d_next_xy,
                                    float* d_back_xy, uint8_t* d_flags, int32_t* d_kept_idx, int32_t* d_n_kept,
                                    double fb_thresh, double border, int32_t cam_w, int32_t cam_h,
                                    const gvx_klt_params* p) {
    if (!c) return GVX_ERR_INVALID;
    gvx_status s = check_klt_params(c, p);
    if (s) return s;
    s = check_batch(c, n_pairs, w, h, d_prev, d_next, n_pts, d_prev_xy, d_next_xy, d_flags, d_kept_idx, d_n_kept);
    if (s) return s;
    if (n_pairs == 0) return GVX_OK;
    if (!d_pyr) return set_err(c, GVX_ERR_INVALID, "bad batch pyramids");
    hipSetDevice(c->device);
    const PyrLayout lay = make_layout(w, h, p->max_level, p->win);
    return klt_batch_on_pyramids(c, lay, n_pairs, w, h, d_prev, d_next, d_pyr, d_pyr + (size_t)lay.bytes * n_pairs,
                                 n_pts, d_prev_xy, d_init_xy, d_next_xy, d_back_xy, d_flags, d_kept_idx, d_n_kept,
                                 fb_thresh, border, cam_w, cam_h, p);
}

gvx_status gvx_klt_fb_batch_dev(gvx_ctx* c, int32_t n_pairs, int32_t w, int32_t h,
                                const uint8_t* d_prev, const uint8_t* d_next, int32_t n_pts,
                                const float* d_prev_xy, float* d_next_xy, float* d_back_xy,
                                uint8_t* d_flags, int32_t* d_kept_idx, int32_t* d_n_kept,
                                double fb_thresh, double border, int32_t cam_w, int32_t cam_h,
                                const gvx_klt_params* p) {
    return gvx_klt_fb_batch_init_dev(c, n_pairs, w, h, d_prev, d_next, n_pts, d_prev_xy, d_next_xy, d_next_xy,
                                     d_back_xy, d_flags, d_kept_idx, d_n_kept, fb_thresh, border, cam_w, cam_h, p);
}

gvx_status gvx_klt_fb_batch(gvx_ctx* c, int32_t n_pairs, int32_t w, int32_t h, const uint8_t* prev,
                            const uint8_t* next, int32_t n_pts, const float* prev_xy, float* next_xy,
                            float* back_xy, uint8_t* flags, int32_t* kept_idx, int32_t* n_kept,
                            double fb_thresh, double border, int32_t cam_w, int32_t cam_h,
                            const gvx_klt_params* p) {
    if (!c) return GVX_ERR_INVALID;
    if (n_pairs <= 0) return GVX_OK;
    if (!prev || !next || (n_pts > 0 && (!prev_xy || !next_xy || !flags || !kept_idx || !n_kept)))
        return set_err(c, GVX_ERR_INVALID, "bad batch pointers");
    hipSetDevice(c->device);
    size_t img = (size_t)w * h * n_pairs;
    size_t pts = sizeof(float) * 2 * (size_t)n_pairs * n_pts;
    size_t np = (size_t)n_pairs * n_pts;
    size_t need = 2 * img + 3 * pts + np + sizeof(int32_t) * (np + n_pairs) + 1024;
    char* d = (char*)scratch(c, "batch_io", need);
    if (!d) return set_err(c, GVX_ERR_OOM, "batch io");
    uint8_t* d_prev = (uint8_t*)d;
    uint8_t* d_next = d_prev + img;
    char* q = (char*)(((uintptr_t)(d_next + img) + 255) & ~(uintptr_t)255);
    float* d_pxy = (float*)q;
    float* d_nxy = (float*)(q + pts);
    float* d_bxy = (float*)(q + 2 * pts);
    int32_t* d_kept = (int32_t*)(q + 3 * pts);
    int32_t* d_nk = d_kept + np;
    uint8_t* d_fl = (uint8_t*)(d_nk + n_pairs);
    hipError_t e = hipMemcpyAsync(d_prev, prev, img, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d_next, next, img, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess && pts) e = hipMemcpyAsync(d_pxy, prev_xy, pts, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess && pts) e = hipMemcpyAsync(d_nxy, next_xy, pts, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "batch H2D");
    gvx_status s = gvx_klt_fb_batch_dev(c, n_pairs, w, h, d_prev, d_next, n_pts, d_pxy, d_nxy, d_bxy,
                                        d_fl, d_kept, d_nk, fb_thresh, border, cam_w, cam_h, p);
    if (s) return s;
    if (pts) {
        e = hipMemcpyAsync(next_xy, d_nxy, pts, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess && back_xy) e = hipMemcpyAsync(back_xy, d_bxy, pts, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(flags, d_fl, np, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(kept_idx, d_kept, sizeof(int32_t) * np, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(n_kept, d_nk, sizeof(int32_t) * n_pairs, hipMemcpyDeviceToHost, c->stream);
        if (e != hipSuccess) return hip_err(c, e, "batch D2H");
    } else if (n_kept) {
        std::memset(n_kept, 0, sizeof(int32_t) * n_pairs);
    }
    return hip_err(c, hipStreamSynchronize(c->stream), "batch sync");
}

}  // extern "C"

namespace gvx {

gvx_status frame_slot(gvx_ctx* c, uint64_t id, int32_t w, int32_t h, const gvx_klt_params* p, Frame** out) {
    gvx_status s = check_klt_params(c, p);
    if (s) return s;
    if (w <= WIN || h <= WIN) return set_err(c, GVX_ERR_INVALID, "frame smaller than the window");
    hipSetDevice(c->device);
    PyrLayout lay = make_layout(w, h, p->max_level, p->win);
    Frame& f = c->frames[id];
    if (!f.pyr || f.lay.bytes < lay.bytes) {
        if (c->capturing) {
            if (!f.pyr) c->frames.erase(id);
            c->capture_failed = true;
            return set_err(c, GVX_ERR_INVALID, "frame %llu needs a (re)allocation during a graph capture",
                           (unsigned long long)id);
        }
        ++c->mem_gen;
        if (f.pyr) {
            sync_all(c);
            hipFree(f.pyr);
            f.pyr = nullptr;
        }
        hipError_t e = hipMalloc(&f.pyr, lay.bytes);
        if (e != hipSuccess) {
            c->frames.erase(id);
            return hip_err(c, e, "hipMalloc(pyramid)");
        }
    }
    f.lay = lay;
    f.w = w;
    f.h = h;
    ++f.gen;  // a new image: an eigenvalue map computed before is stale
    *out = &f;
    return GVX_OK;
}

}  // namespace gvx
