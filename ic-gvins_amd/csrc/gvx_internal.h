// gvx_internal.h -- shared host-side definitions of libgvx (not part of the ABI).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "gvx.h"

namespace gvx {

// Pyramid storage (DESIGN.md "HBM layout"): every level is stored
// with a PAD-pixel BORDER_REFLECT_101 ring so that LK window gathers (including
// the Scharr halo and 16-byte aligned row loads) never leave the allocation.
// OpenCV pads by winSize (21); the extra ring beyond 21 px is never read by a
// valid computation.
constexpr int PAD = 32;
constexpr int MAX_LEVELS = 7;
constexpr int WIN = 21;  // the device LK kernel is specialised for 21x21

struct PyrLayout {
    int32_t nlev;                  // levels built (maxLevel actually used + 1)
    int32_t w[MAX_LEVELS], h[MAX_LEVELS];
    int32_t pitch[MAX_LEVELS];     // bytes per padded row (multiple of 64)
    int64_t off[MAX_LEVELS];       // byte offset of padded (-PAD,-PAD) of level l
    int64_t bytes;                 // bytes per image pyramid (multiple of 256)
};

// buildOpticalFlowPyramid's level count rule (stop when the next level would be
// <= win on either side) -- identical for both images of a pair.
PyrLayout make_layout(int w, int h, int max_level, int win);

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    bool fresh = false;  // (re)allocated since a caller last cleared it (zero-initialised state)
};

struct Frame {
    PyrLayout lay;
    uint8_t* pyr = nullptr;  // device
    int w = 0, h = 0;
    // the detection's eigenvalue map of this frame (gvx_frame_eig_dev), for the
    // block grid of eig_key (block size, 0 = none)
    float* eig = nullptr;
    size_t eig_bytes = 0;
    long eig_key = 0;
    uint64_t gen = 0, eig_gen = 0;  // pyramid writes so far; the write the eig map belongs to
};

struct ProfEntry {
    double ms = 0;
    int64_t launches = 0;
};

}  // namespace gvx

struct gvx_ctx {
    int device = 0;
    int n_cu = 256;  // compute units (persistent-grid sizing)
    hipStream_t stream = nullptr;
    // gvx_branch_begin / _end / _join: `stream` points at `side` inside a branch;
    // `main` is the context's own stream (the one gvx_sync and captures use)
    hipStream_t main = nullptr, side = nullptr;
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
    bool in_branch = false, branch_open = false;  // enqueuing on side / a recorded branch not yet joined
    std::string err;
    std::unordered_map<uint64_t, gvx::Frame> frames;
    // scratch (grown on demand, never shrunk)
    std::map<std::string, gvx::DevBuf> dev;
    std::map<std::string, gvx::DevBuf> pinned;
    // bumped whenever device memory a captured graph may reference is freed or
    // moved (scratch growth, a frame pyramid reallocated or dropped): a graph
    // captured under another generation refuses to launch
    uint64_t mem_gen = 0;
    bool capturing = false;
    uint64_t capture_gen = 0;
    // a call inside the open capture failed for want of a (re)allocation:
    // gvx_capture_end refuses the graph
    bool capture_failed = false;
    // gvx_set_marg_solver
    int32_t marg_solver = GVX_MARG_SOLVER_FAST;
    // gvx_set_preint_path (GVX_PREINT_ONEPHASE=1 at creation: the single kernel)
    int32_t preint_path = GVX_PREINT_PATH_AUTO;
    // factor sets created with a device result buffer and a D2H copy per prepare
    // (GVX_FACTORSET_D2H=1 at creation; A/B against the mapped host buffer)
    bool factorset_d2h = false;
    // gvx_track_frame_dev: what the detection constants in "trk_static" were
    // built for (the buffer itself and the geometry)
    struct TrackStatic {
        const void* buf = nullptr;
        size_t bytes = 0;
        int64_t w = 0, h = 0, max_features = 0, block_size = 0;
        bool operator==(const TrackStatic& o) const {
            return buf == o.buf && bytes == o.bytes && w == o.w && h == o.h && max_features == o.max_features &&
                   block_size == o.block_size;
        }
    } track_static;
    // profiling
    bool prof = false;
    bool prof_markers = false;  // GVX_PROF_MARKERS=1 at creation (launch_timed)
    // batch LK (three points per wave): levels per phase of klt_phase_kernel, 0 =
    // one wave runs the whole chain (klt_kernel); GVX_KLT_LPP at creation
    int klt_lpp = 0;
    int klt_super = 4096;  // groups per superchunk of klt_phase_kernel (GVX_KLT_SUPER)
    // pyramid pass (stream_kernel): waves per workgroup (1 or 4) and work order
    // (1: edge strips first); GVX_PYR_WPB / GVX_PYR_ORDER at creation (A/B)
    int pyr_wpb = 1, pyr_order = 0;
    // small fwd + bwd launches (one point per wave) compact inside the LK launch
    // instead of a compact_kernel launch; GVX_FUSED_COMPACT=0 at creation: off (A/B)
    bool fused_compact = true;
    // GVX_SIDE_LOW_PRIO=1 at creation: the branch stream at the lowest priority,
    // the context stream at the highest (work on the branch fills the gaps); 2:
    // the other way round; 0 (default): both at the default priority
    int side_low_prio = 0;
    std::map<std::string, gvx::ProfEntry> prof_acc;
    struct Pending {
        std::string fam;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> event_pool;
};

namespace gvx {

gvx_status set_err(gvx_ctx* c, gvx_status s, const char* fmt, ...);
gvx_status hip_err(gvx_ctx* c, hipError_t e, const char* what);
void* scratch(gvx_ctx* c, const std::string& name, size_t bytes);
// both streams of the context (the side branch's too): before memory is freed
void sync_all(gvx_ctx* c);   // device
void* pinned(gvx_ctx* c, const std::string& name, size_t bytes);    // pinned host
// the cached frame `id` sized for (w, h, p) (allocated or grown; refuses to
// reallocate during a graph capture)
gvx_status frame_slot(gvx_ctx* c, uint64_t id, int32_t w, int32_t h, const gvx_klt_params* p, Frame** out);

// Profiling brackets around a kernel family launch (no-ops when disabled).
void prof_begin(gvx_ctx* c, const char* fam, hipEvent_t* a);
void prof_end(gvx_ctx* c, const char* fam, hipEvent_t a);
void prof_drain(gvx_ctx* c);
hipEvent_t prof_event(gvx_ctx* c);
void prof_push(gvx_ctx* c, const char* fam, hipEvent_t a, hipEvent_t b);
// A kernel launch on the context stream; with profiling on, timed by events
// attached to the dispatch itself (hipExtLaunchKernel: the kernel's own start /
// stop, as rocprofv3 sees it) instead of markers recorded around the launch,
// which add the dispatch gaps (~2 us, r03 v29 trace against the bench line).
template <typename... Args, typename F = void (*)(Args...)>
hipError_t launch_timed(gvx_ctx* c, const char* fam, F kernel, dim3 grid, dim3 block, uint32_t shmem,
                        Args... args) {
    if (!c->prof || c->capturing) {
        hipLaunchKernelGGL(kernel, grid, block, shmem, c->stream, args...);
        return hipGetLastError();
    }
    hipEvent_t a = prof_event(c), b = prof_event(c);
    if (c->prof_markers) {
        hipEventRecord(a, c->stream);
        hipLaunchKernelGGL(kernel, grid, block, shmem, c->stream, args...);
        hipEventRecord(b, c->stream);
    } else {
        hipExtLaunchKernelGGL(kernel, grid, block, shmem, c->stream, a, b, 0, args...);
    }
    const hipError_t e = hipGetLastError();
    prof_push(c, fam, a, b);
    return e;
}


// ---- kernel launchers (klt.hip) ----
// Build pyramids for n_img images (h x w, row stride `stride` bytes, image i at
// src + i*img_stride) into dst + i*lay.bytes: levels >= 1 always; the padded
// level-0 copy only when write_l0 (otherwise level 0 stays the caller's image).
// src_b (optional): images n_a .. n_img-1 come from src_b + (i - n_a)*img_stride
// instead (the prev and next frames of a batch built in one launch per kernel).
// l0_in_slot: level 0 with its ring is already in dst's padded level-0 slot
// (written there by the CLAHE pass); only levels >= 1 are built, from it.
hipError_t launch_build_pyramids(gvx_ctx* c, const uint8_t* src, int64_t img_stride, int stride,
                                 int n_img, const PyrLayout& lay, uint8_t* dst, bool write_l0,
                                 const uint8_t* src_b = nullptr, int n_a = 0, bool l0_in_slot = false);

// Workgroups are dispatched to the 8 XCDs round-robin by id (each XCD has its
// own L2).  xcd_swizzle maps the dispatch id to a logical id so that XCD k runs
// the contiguous logical range [k*per, (k+1)*per): neighbouring work (points of
// one frame pair, adjacent image tiles) shares one L2.  The grid must hold
// 8*per workgroups; logical ids >= n are idle.
#ifdef GVX_KLT_TRACE
// Diagnostic builds only (EXTRA=-DGVX_KLT_TRACE tools/variant.sh): a wave stores
// {wave id, start, end (s_memrealtime, 100 MHz), HW_ID | XCC_ID << 32} to
// buf[4 * id] when it leaves (tools/lk_residency.py, tools/pyr_residency.py).
// The product build compiles none of this.
struct WaveStamp {
    uint64_t* buf;
    uint64_t t0;
    __device__ explicit WaveStamp(uint64_t* b) : buf(b) { t0 = __builtin_amdgcn_s_memrealtime(); }
    __device__ ~WaveStamp() {
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // XCC_ID
        if (buf && (threadIdx.x & 63) == 0) {
            const uint64_t id = (uint64_t)blockIdx.x * blockDim.x / 64 + (threadIdx.x >> 6);
            buf[4 * id] = id;
            buf[4 * id + 1] = t0;
            buf[4 * id + 2] = t1;
            buf[4 * id + 3] = (uint64_t)hw | ((uint64_t)xcc << 32);
        }
    }
};
#endif

constexpr int N_XCD = 8;
__host__ __device__ inline int xcd_per(int n) { return (n + N_XCD - 1) / N_XCD; }
__device__ inline int xcd_swizzle(int b, int n) { return (b % N_XCD) * xcd_per(n) + b / N_XCD; }

struct KltArgs {
    int32_t n_pairs, n_pts;
    int32_t max_iter;
    double crit_eps;         // eps*eps (double, like OpenCV criteria.epsilon)
    float min_eig;
    int32_t use_initial_flow;
    int32_t accum;           // GVX_LK_ACCUM_*
    int32_t mode;            // 0: single LK, 1: fwd + bwd + FB
    double fb_thresh, border;
    int32_t cam_w, cam_h;
    // device-resident point count (n_pairs == 1 only): the launch is sized for
    // n_pts points (the capacity), the kernel tracks min(*n_dev, n_pts)
    const int32_t* n_dev = nullptr;
    // initial flow read from here instead of next_xy (which is then output only)
    const float* init_xy = nullptr;
    // compaction inside the LK launch (one point per wave, mode 1, no n_dev):
    // per pair ceil(n_pts / 64) keep-bit words and an arrival count, zero at
    // launch; the last wave of a pair writes kept_idx / n_kept (compact_kernel's
    // result) and zeroes them again (klt.hip fused_compact)
    unsigned long long* cmask = nullptr;
    int32_t* kept_idx = nullptr;
    int32_t* n_kept = nullptr;
};

// Level 0 of pair i: prev plane at prev + i*prev_stride, pixel (x, y) at byte
// o0 + y*pitch + x, likewise next.  raw = 1: the caller's unpadded images
// (o0 = 0; border windows are gathered with REFLECT_101); raw = 0: the padded
// level-0 slot of a pyramid (base at the ring's corner, o0 = PAD*pitch + PAD).
struct Level0 {
    const uint8_t* prev;
    const uint8_t* next;
    int64_t prev_stride, next_stride;
    int32_t o0, pitch, raw;
};

// Pyramid (levels >= 1) of pair i: prev at pyr_prev + i*prev_pair_stride, next
// at pyr_next + i*next_pair_stride.
hipError_t launch_klt(gvx_ctx* c, const KltArgs& a, const PyrLayout& lay, const uint8_t* pyr_prev,
                      const uint8_t* pyr_next, int64_t prev_pair_stride, int64_t next_pair_stride,
                      const Level0& l0, const float* prev_xy, float* next_xy, float* back_xy, uint8_t* flags,
                      float* err);
hipError_t launch_compact(gvx_ctx* c, int n_pairs, int n_pts, const uint8_t* flags, int32_t* kept_idx,
                          int32_t* n_kept);
// fwd + bwd + FB (a.mode must be 1) and the compaction: inside the LK launch
// when it runs one point per wave (c->fused_compact), else launch_klt +
// launch_compact
hipError_t launch_klt_compact(gvx_ctx* c, KltArgs a, const PyrLayout& lay, const uint8_t* pyr_prev,
                              const uint8_t* pyr_next, int64_t prev_pair_stride, int64_t next_pair_stride,
                              const Level0& l0, const float* prev_xy, float* next_xy, float* back_xy,
                              uint8_t* flags, float* err, int32_t* kept_idx, int32_t* n_kept);

// ---- clahe.hip ----
// CLAHE_Impl::apply geometry for an h x w 8-bit image (oracle/clahe.c).
struct ClaheGeom {
    int32_t w, h, tiles_x, tiles_y;
    int32_t tw, th;      // tile size (of the REFLECT_101-extended LUT source)
    int32_t clip;        // clipLimit in pixels (0: no clipping)
    float lut_scale;     // 255.f / (tw*th)
};
ClaheGeom clahe_geometry(int w, int h, double clip_limit, int tiles_x, int tiles_y);
// n images; lut: n*tiles*256 bytes scratch; hist_img (nullable): n*256 u32
// scratch for the histogram check, whose means go to hist_mean (device).
// src_index (n == 1): the source is src + (*src_index) * img_stride, picked on the
// device, the index clamped to [0, n_src - 1]; ring: dst is pixel (0,0) of a
// padded level (PAD ring written too)
hipError_t launch_clahe(gvx_ctx* c, int n, const ClaheGeom& g, const uint8_t* src, int64_t img_stride,
                        int stride, uint8_t* dst, int64_t dst_img_stride, int dst_stride, uint8_t* lut,
                        uint32_t* hist_img, double* hist_mean, const int32_t* src_index = nullptr,
                        int n_src = 0, int ring = 0, int chan = 1, uint8_t* gray = nullptr);
// gray scratch of launch_clahe for chan 3: n images of clahe_gray_pitch(w) x h bytes
inline int clahe_gray_pitch(int w) { return (w + 63) & ~63; }

// ---- aux_factors.hip ----
// residuals of a small factor kind (0: unknown kind); *P block size, *NC constants per factor
int small_factor_dims(int kind, int* P, int* NC);
hipError_t launch_small_factor(gvx_ctx* c, int kind, int n, const double* consts, const double* params,
                               const int32_t* offs, double* residuals, double* jacobians);
// blk = {size[nb], index[nb], xoff[nb]}
hipError_t launch_marg_factor(gvx_ctx* c, int r, int nb, const int32_t* blk, const double* x0, const double* x,
                              const double* J0, const double* e0, double* residuals, double* jacobians);

// ---- marg.hip ----
constexpr int GVX_EIG_MAX_N = 512;  // largest SelfAdjointEigenSolver the one-workgroup kernel takes
// One lower block pair (row block P at row0, column block Q at col0) of H0, or
// (col0 = -1, lq = 1) one block of b0; its contributions are contrib[c0 .. c1).
struct MargPairRec {
    int32_t row0, col0, lp, lq, c0, c1;
};
struct MargLaunch {
    int n_pairs, n_bvec;              // H0 records first, then the b0 records
    const MargPairRec* pairs;         // device
    const int4* contrib;              // device
    int n_fac;
    const int32_t* nres;              // device (loss only)
    const int64_t* res_off;           // device (loss only)
    const double* loss;               // device, nullable
    double* sr;                       // device scratch [n_fac]
    const double* data;               // device: the evaluated residual blocks
    int L, m;
    double *H0, *b0, *V1, *w1, *Hinv, *T, *Hp, *bp, *V2, *w2, *hc;
    int* info;                        // device [2]: Hmm and Hp eigen-solver status
    double *J0, *e0;
    // GVX_MARG_SOLVER_*; FAST: Cholesky factors Lm (m x m), Lp (r x r), X = Lm^-1
    // [Hmr | bm] (m x (r + 1) row-major) and the two check flags chol[2] (device)
    int solver;
    double *Lm, *Lp, *X;
    int* chol;
    // FAST: H0 / b0 from contribution chunks (chunk = {record, c0, c1, partial
    // offset}; recpart[k] = {first partial, chunks} of record k), partial sums in part
    int n_chunks;
    const int4* chunks;
    const int2* recpart;
    double* part;
    // LM step: Hee is diagonal (every eliminated block has one local parameter and
    // no factor couples two of them): Lm holds only its diagonal, no m limit
    int diag_e;
};
hipError_t launch_marginalize(gvx_ctx* c, const MargLaunch& p);
// constructEquation alone (H0 = sum J^T J, b0 = -sum J^T e; chunked when p.chunks)
hipError_t launch_h0(gvx_ctx* c, const MargLaunch& p);
// ---- dense.hip (fp64 Cholesky kernels; gate: skipped unless *gate == 0) ----
hipError_t launch_potrf(gvx_ctx* c, int n, const double* A, int lda, double shift, double* L, int* fail,
                        const int* gate);
hipError_t launch_trsv(gvx_ctx* c, int n, const double* L, int nrhs, const double* B, long ldb, double* X, int ldx,
                       bool neg, const int* gate);
hipError_t launch_schur_chol(gvx_ctx* c, int L, int m, const double* H0, const double* b0, const double* X,
                             double* Hp, double* bp, const int* gate);
hipError_t launch_lin_chol(gvx_ctx* c, int r, const double* Lp, double* J0, double* eval, const int* gate);
// (J^T J + diag(D^2)) delta = -J^T r with the first m local parameters eliminated
// (DENSE_SCHUR): p's lists / H0 / b0 / Lm / Lp / X / chol (2 flags, zeroed by the
// caller: potrf failures of Hee + D and of S); S r x r, bs r, tmp >= 2 m + r
hipError_t launch_lm_step(gvx_ctx* c, const MargLaunch& p, const double* D, double* delta, double* S, double* bs,
                          double* tmp);
// SelfAdjointEigenSolver of the lower triangle of src (ld lds): V n x n, w n, hc n scratch, info 1 int;
// ts (nullable, diagnostics): 7 u64, wall-clock stamps (100 MHz) of the solver's phases + QR iterations
hipError_t launch_sym_eigen(gvx_ctx* c, int n, const double* src, int lds, double* V, double* w, double* hc,
                            int* info, unsigned long long* ts = nullptr);

// ---- fmat.hip ----
// cv::findFundamentalMat(FM_RANSAC) per point set: set i = points off[i] .. off[i+1]
hipError_t launch_fm_ransac(gvx_ctx* c, int n_prob, const int32_t* off, const float* p1, const float* p2,
                            double thresh, double confidence, int max_iters, uint8_t* mask, double* F,
                            int32_t* result, unsigned long long* ts = nullptr);

// ---- ins.hip ----
hipError_t launch_ins(gvx_ctx* c, const gvx_ins_config& cfg, int n_chain, const gvx_imu* imu, const int32_t* off,
                      const gvx_state* state0, gvx_state* states);

// ---- camera.hip ----
struct CamArgs {
    gvx_camera cam;
    double M[9];  // r_cur_pre (PREDICT), pose R (PROJECT), R1^T R0 (PARALLAX)
    double t[3];  // pose t (PROJECT)
    double dt;    // VELOCITY
    int32_t n;
};
hipError_t launch_camera(gvx_ctx* c, int op, const CamArgs& a, const void* in0, const void* in1, void* out);

// ---- preint.hip / factors.hip ----
hipError_t launch_preint(gvx_ctx* c, int variant, const gvx_imu_params& prm, int n_seg,
                         const gvx_imu* imu, const int32_t* seg_off, const gvx_state* state0,
                         const double* iewn, gvx_preint_result* out, double* pn,
                         bool* sqrt_info_done = nullptr);  // set when the covariance pass formed sqrt_info
// both factor kinds of a small window in one launch (factors.hip window_factor_kernel)
hipError_t launch_window_factors(gvx_ctx* c, int n_r, const gvx_reproj_const* cs, const int32_t* roffs, double* rres,
                                 double* rjac, int n_p, const gvx_preint_result* pre, const double* pn,
                                 const int32_t* pn_off, const int32_t* poffs, double* pres, double* pjac,
                                 const double* params);
int window_factor_blocks(int n_r, int n_p);
hipError_t launch_reproj(gvx_ctx* c, int n, const gvx_reproj_const* cs, const double* params,
                         const int32_t* offs, double* res, double* jac);
hipError_t launch_sqrt_info(gvx_ctx* c, int n, gvx_preint_result* pre);
hipError_t launch_preint_factor(gvx_ctx* c, int n, const gvx_preint_result* pre, const double* pn,
                                const int32_t* pn_off, const double* params, const int32_t* offs,
                                double* res, double* jac);

// ---- detect.hip ----
struct DetectLaunch {
    int w, h;
    const uint8_t* img0;  // padded level 0 at image (0,0)
    int pitch;
    // circle mask
    const int2* centers;
    int n_circles, radius, fill_mask;
    const int* hw;        // half-width per row offset 0..radius (-1 = none)
    uint8_t* mask;        // w x h
    // blocks
    const int4* rois;     // (x0, y0, rw, rh) per block
    const int* blk_ids;   // active blocks (want > 0)
    int n_active, n_blocks, max_rw, max_rh;
    const int* want;      // maxCorners per block
    int64_t eig_stride;
    float* eig;
    unsigned long long* cand;
    int2* corners;
    int* ncorner;
    int max_per_block;
    double quality;
    float min_dist;
    float sc, sc2;        // Sobel scale 1/(4*3*255) and 2x
    const float* gmask;   // 11x11 cornerSubPix weights
    int max_iters;
    double eps2;
    float2* out;
    // device-resident counts (gvx_track_frame_dev): circles, active blocks and a
    // skip flag read by the kernels; nullptr for host-counted calls
    const int* n_circles_dev = nullptr;
    const int* n_active_dev = nullptr;
    const int* skip_dev = nullptr;
};
hipError_t launch_detect(gvx_ctx* c, const DetectLaunch& d);
// cornerMinEigenVal tiles of every block (block k at eig + k * eig_stride, ROI
// raster order): the part of the detection that depends on the frame alone
hipError_t launch_eig_all(gvx_ctx* c, int n_blocks, int max_rw, int max_rh, const uint8_t* img0, int pitch,
                          const int4* rois, int64_t eig_stride, float* eig, float sc, float sc2);
// The tracking path's per-block detection (select_track_kernel): counts, early
// exit, the LDS circle mask and the selection in one workgroup per block.
constexpr int TS_MAX_POINTS = 1024;        // tracker capacity the kernel's LDS holds
constexpr size_t TS_MAX_BITMAP = 32 * 1024;  // ROI mask bitmap bytes
struct TrackSelect {
    int bcols, col, row, maxpb, max_features, cap, radius;
    const int32_t* n;       // tracked points before the FB update
    const uint8_t* flags;   // LK flags (bit 2 = kept) or nullptr: pts[0, n) as they are
    const float* next_xy;   // tracked positions (flags != nullptr)
    const float* pts;       // the point list (flags == nullptr)
    const int4* rois;
    const int* hw;          // circle half-width per row offset 0..radius
    const float* eig;
    int64_t eig_stride;
    unsigned long long* cand;
    int2* corners;
    int* ncorner;
    int max_per_block;
    double quality;
    float min_dist;
    const uint8_t* img0;
    int pitch;
    const float* gmask;
    int max_iters;
    double eps2;
    float2* out;
    // per block {fkey of the max over the mask, candidate count} from the tiles'
    // scan (eig_track_kernel), zero between frames; nullptr: the selection scans
    // the whole ROI itself (an eigenvalue map computed elsewhere)
    unsigned* sel;
};
size_t select_track_lds(int max_rw, int max_rh);
// the eigenvalue tiles of the blocks that detect this frame (a.eig is written)
hipError_t launch_eig_track(gvx_ctx* c, int n_blocks, int max_rw, int max_rh, const TrackSelect& a, float sc,
                            float sc2);
hipError_t launch_select_track(gvx_ctx* c, int n_blocks, int max_rw, int max_rh, const TrackSelect& a);

// ---- track.hip (gvx_track_frame_dev, gvx_copy_dev) ----
hipError_t launch_copy(gvx_ctx* c, void* dst, const void* src, size_t bytes);
hipError_t launch_copy_indexed(gvx_ctx* c, void* dst, const void* src_base, size_t bytes, const int32_t* index,
                               int n_src);
hipError_t launch_index_advance(gvx_ctx* c, int32_t* index, int32_t delta);
hipError_t launch_track_record(gvx_ctx* c, const float* pts, const int32_t* n, int cap, float* tracks,
                               int32_t* counts, int32_t* frame, int max_frames);
// the device tracker state after the forward/backward LK: keep-flag compaction,
// pts <- next[kept], vel <- next[kept] - pts[kept], init <- pts + vel, n <- kept
hipError_t launch_track_update(gvx_ctx* c, int cap, int32_t* n, const uint8_t* flags, const float* next_xy,
                               float* pts, float* vel, float* init, int32_t* kept_out);
struct DetectPrep {
    int bcols, brows, col, row, maxpb, max_features;
    const float* pts;
    const int32_t* n;
    // the reduceVector update of the FB result first, in the same launch (track
    // frames): flags / next_xy -> pts (compacted), vel, init, kept_out, *n
    int update_cap;  // 0: no update
    const uint8_t* flags;
    const float* next_xy;
    float* upd_pts;
    float* vel;
    float* init;
    int32_t* kept_out;
    int32_t* n_upd;
    int* want;
    int* blk_ids;
    int* n_active;
    int2* centers;
    int* n_circles;
    int* skip;
    int* ncorner;
};
hipError_t launch_detect_prep(gvx_ctx* c, const DetectPrep& p);
// append the detected corners (block order, block origin added) up to
// max_features: pts / init = corner, vel = 0, n grows; corners_out (nullable)
// receives every corner and *n_corners_out their count (-1 when skipped)
// rec (nullable): then append the track list to the per-frame record (as
// launch_track_record) in the same launch
struct TrackRecord {
    float* tracks;
    int32_t* counts;
    int32_t* frame;
    int max_frames, cap;
};
// the tracking path's last launch: update (update_cap > 0), the early exit from
// the kept count, the corners appended, the record (rec.tracks != nullptr)
struct TrackMerge {
    int bcnt, bcols, col, row, maxpb, max_features;
    int out_stride;  // corner slots per block in out (max(maxpb, 1))
    int update_cap;
    const uint8_t* flags;
    const float* next_xy;
    float *pts, *vel, *init;
    int32_t* kept_out;
    int32_t* n;
    const int* ncorner;
    const float2* out;
    float* corners_out;
    int32_t* n_corners_out;
    TrackRecord rec;
};
hipError_t launch_track_merge(gvx_ctx* c, const TrackMerge& m);
hipError_t launch_detect_merge(gvx_ctx* c, int bcnt, int bcols, int col, int row, int maxpb, int max_features,
                               const int* skip, const int* ncorner, const float2* out, float* pts, float* vel,
                               float* init, int32_t* n, float* corners_out, int32_t* n_corners_out,
                               const TrackRecord* rec = nullptr);

// Staging layout for host-pointer API calls: ONE list of slices both sizes the
// buffer and carves it (256-byte aligned, in declaration order), so the two can
// never disagree.  add() registers the device pointer (and, optionally, the
// pinned-host twin at the same offset); bind() assigns every registered pointer
// once the buffers exist.  A zero count still takes one aligned slot, so the
// slices stay distinct and in order (callers size contiguous ranges with
// pointer differences).
class Staging {
  public:
    template <class T>
    void add(size_t count, T** dev, T** host = nullptr) {
        items_.push_back({total_, reinterpret_cast<void**>(dev), reinterpret_cast<void**>(host)});
        total_ += (std::max<size_t>(count, 1) * sizeof(T) + 255) & ~size_t(255);
    }
    size_t bytes() const { return total_ ? total_ : 256; }
    void bind(void* dev_base, void* host_base = nullptr) const {
        for (const Item& it : items_) {
            *it.dev = static_cast<char*>(dev_base) + it.off;
            if (it.host) *it.host = host_base ? static_cast<char*>(host_base) + it.off : nullptr;
        }
    }

  private:
    struct Item {
        size_t off;
        void** dev;
        void** host;
    };
    std::vector<Item> items_;
    size_t total_ = 0;
};

}  // namespace gvx
