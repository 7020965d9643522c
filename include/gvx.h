/*
 * gvx.h -- C ABI of the MI355X-native IC-GVINS front end (libgvx.so).
 *
 * Plain C types only (no HIP, torch or C++ types in any signature).  Every call
 * returns gvx_status (0 = OK, negative = error; gvx_last_error() has the text);
 * no exception crosses the ABI.  Calls are synchronous unless their name ends in
 * _dev (device pointers, enqueued on the context stream; gvx_sync() waits).
 * One context per host thread, or serialise calls on a shared context.
 *
 * Each entry point names the reference interface it replaces
 * (paths relative to /root/reference/ic_gvins/ic_gvins/).
 */
#ifndef GVX_H
#define GVX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t gvx_status;
enum {
    GVX_OK = 0,
    GVX_ERR_INVALID = -1,   /* bad argument (the reference would throw cv::Exception / assert) */
    GVX_ERR_NO_DEVICE = -2, /* no gfx950 device / HIP runtime unavailable */
    GVX_ERR_HIP = -3,       /* a HIP runtime call failed */
    GVX_ERR_OOM = -4,       /* device or host allocation failed */
    GVX_ERR_NOT_FOUND = -5, /* unknown frame id */
    GVX_ERR_UNSUPPORTED = -6,
    GVX_ERR_NUMERIC = -7    /* a factorisation met a non-positive pivot (gvx_schur_solve: outputs NaN) */
};

typedef struct gvx_ctx gvx_ctx;

/* ---------------------------------------------------------------- context */
gvx_status gvx_create(int32_t device, gvx_ctx** out);
void gvx_destroy(gvx_ctx* ctx);
const char* gvx_status_string(gvx_status s);
const char* gvx_last_error(const gvx_ctx* ctx);
gvx_status gvx_sync(gvx_ctx* ctx);
/* The hipStream_t all work of this context is enqueued on (opaque). */
void* gvx_get_stream(gvx_ctx* ctx);
/* Library version string, e.g. "gvx 0.1 gfx950". */
const char* gvx_version(void);

/* Per-kernel-family device time, accumulated with HIP events on the context
   stream while enabled (used by bench.py's roofline).  family: "pyramid",
   "klt", "compact", "detect", "preint", "reproj", "preint_factor". */
gvx_status gvx_profile_enable(gvx_ctx* ctx, int32_t on);
gvx_status gvx_profile_read(gvx_ctx* ctx, const char* family, double* total_ms, int64_t* launches);
gvx_status gvx_profile_reset(gvx_ctx* ctx);

/* ---------------------------------------------------------------- hipGraphs */
/* Capture what this context enqueues between gvx_capture_begin and
   gvx_capture_end (stream capture of the context stream) into a graph that
   gvx_graph_launch replays with one launch: one frame pair per graph launch
   (BASELINE configs[1]) instead of one host call per kernel.
   Only *_dev entry points may be captured, after one uncaptured call with the
   same sizes (so no scratch buffer grows during capture), with profiling off.
   A captured graph holds raw pointers to the context's scratch buffers and to
   the cached frame pyramids.  Any later call that reallocates them (a scratch
   buffer growing for larger sizes, gvx_frame_put with a bigger layout,
   gvx_frame_drop) invalidates every graph of the context: gvx_graph_launch then
   refuses with GVX_ERR_INVALID instead of touching freed memory.  Calls that
   would reallocate during an open capture fail (GVX_ERR_INVALID / GVX_ERR_OOM)
   and gvx_capture_end then refuses the graph. */
typedef struct gvx_graph gvx_graph;
gvx_status gvx_capture_begin(gvx_ctx* ctx);
gvx_status gvx_capture_end(gvx_ctx* ctx, gvx_graph** out);
/* End an open capture and discard it (a call inside it failed): closes an open
   branch, ends the stream capture and destroys the partial graph, so the context
   is usable again.  A no-op when no capture is open. */
gvx_status gvx_capture_abort(gvx_ctx* ctx);
gvx_status gvx_graph_launch(gvx_ctx* ctx, const gvx_graph* g);
void gvx_graph_destroy(gvx_graph* g);
/* Device-to-device copy on the context stream (capturable: e.g. the initial
   flow copied into next_xy before each replay).  A copy kernel on the compute
   queue (no DMA engine hand-off inside a graph). */
gvx_status gvx_copy_dev(gvx_ctx* ctx, void* d_dst, const void* d_src, size_t bytes);
/* One side branch of the context's stream: the *_dev calls between
   gvx_branch_begin and gvx_branch_end are enqueued on a second stream that
   first waits for everything enqueued before gvx_branch_begin; the calls after
   gvx_branch_end go to the context stream again, concurrently with the branch,
   until gvx_branch_join makes the context stream wait for the branch.  Inside a
   capture the branch becomes a parallel path of the graph (the sequence replay
   preprocesses frame t+1 beside frame t's tracking).  Work of the two paths
   must not share scratch buffers or frame slots.  One branch at a time; the
   first gvx_branch_begin of a context must not be inside a capture (it creates
   the stream); a capture must not begin or end with a branch open (gvx_sync
   also completes an ended branch). */
gvx_status gvx_branch_begin(gvx_ctx* ctx);
gvx_status gvx_branch_end(gvx_ctx* ctx);
gvx_status gvx_branch_join(gvx_ctx* ctx);

/* ------------------------------------------------------------------ KLT  */
/* cv::calcOpticalFlowPyrLK arguments as used at tracking/tracking.cc:385-393:
   Size(21,21), maxLevel TRACK_PYRAMID_LEVEL=3 (tracking/tracking.h:113),
   TermCriteria(COUNT+EPS, 30, 0.01), OPTFLOW_USE_INITIAL_FLOW, minEig 1e-4. */
typedef struct {
    int32_t win;              /* window side; the device path supports 21 */
    int32_t max_level;        /* <= 6 */
    int32_t max_iter;         /* TermCriteria COUNT, clamped to [0,100] like OpenCV */
    double eps;               /* TermCriteria EPS (squared internally) */
    int32_t use_initial_flow; /* OPTFLOW_USE_INITIAL_FLOW */
    float min_eig;            /* minEigThreshold */
    int32_t accum;            /* GVX_LK_ACCUM_*: order of the 21x21 window sums */
} gvx_klt_params;
/* Window-sum order of LK's structure tensor A and mismatch vector b
   (LKTrackerInvoker::operator()):
   EXACT      exact integer sums rounded once to fp32 (default; machine
              independent, the restatement's documented order);
   F32_SCALAR OpenCV 4.x's scalar loop: one fp32 accumulator per sum, each
              int32 product converted to float and added in row-major order
              (non-SIMD builds);
   F32_SIMD4  OpenCV 4.x's CV_SIMD128 path (x86 builds): pixels 0..15 of each
              row in 4-lane fp32 accumulators (lane x mod 4), pixels 16..20 in
              the scalar accumulator, the lanes reduced and added last.
   All three are bit-exact against oracle/klt.c's orc_set_lk_accum modes. */
#define GVX_LK_ACCUM_EXACT 0
#define GVX_LK_ACCUM_F32_SCALAR 1
#define GVX_LK_ACCUM_F32_SIMD4 2
void gvx_klt_params_default(gvx_klt_params* p);

/* Upload one gray u8 frame (Frame::image() after CLAHE, tracking/frame.h:62-64)
   and build its padded pyramid on the device once; replaces the per-call
   buildOpticalFlowPyramid inside each of the four cv::calcOpticalFlowPyrLK calls
   per frame (tracking/tracking.cc:385,390,487,493).  Re-putting an id replaces it. */
gvx_status gvx_frame_put(gvx_ctx* ctx, uint64_t id, const uint8_t* gray, int32_t w, int32_t h,
                         int32_t stride, const gvx_klt_params* p);

/* The same from an image already in device memory (d_gray, row stride in
   bytes): the pyramid build is enqueued on the context stream and the call
   returns without waiting (sequence replay with frames resident in HBM). */
gvx_status gvx_frame_put_dev(gvx_ctx* ctx, uint64_t id, const uint8_t* d_gray, int32_t w, int32_t h,
                             int32_t stride, const gvx_klt_params* p);
gvx_status gvx_frame_drop(gvx_ctx* ctx, uint64_t id);

/* One cv::calcOpticalFlowPyrLK(prev, next, prevPts, nextPts, status, err, ...)
   on cached frames.  next_xy is in/out when use_initial_flow.  n may be 0. */
gvx_status gvx_klt(gvx_ctx* ctx, uint64_t prev_id, uint64_t next_id, const float* prev_xy,
                   float* next_xy, uint8_t* status, float* err, int32_t n, const gvx_klt_params* p);

/* Fused replacement of tracking/tracking.cc:380-408 (and :482-511):
   forward LK prev->next with initial flow next_xy, backward LK next->prev with
   initial flow prev_xy, keep = st_f && st_b && !isOnBorder(next) &&
   ptsDistance(back, prev) < fb_thresh (tracking.cc:396-403, :841-849), then the
   order-preserving reduceVector compaction (tracking.cc:831-839) as an index
   list.  Outputs: next_xy (forward result), back_xy, status_fwd, status_bwd,
   keep[n], kept_idx[*n_kept].  border = 5.0, fb_thresh = 0.5 in the reference;
   cam_w/cam_h = camera_->width()/height(). Any output pointer except next_xy and
   n_kept may be NULL. */
gvx_status gvx_klt_fb(gvx_ctx* ctx, uint64_t prev_id, uint64_t next_id, const float* prev_xy,
                      float* next_xy, float* back_xy, uint8_t* status_fwd, uint8_t* status_bwd,
                      uint8_t* keep, int32_t* kept_idx, int32_t* n_kept, int32_t n,
                      double fb_thresh, double border, int32_t cam_w, int32_t cam_h,
                      const gvx_klt_params* p);

/* Batched frame-pair unit, device pointers, async on the context
   stream: for each pair i, build the pyramids of prev[i] and next[i]
   (h x w u8, tightly packed, pair-major), run gvx_klt_fb on n_pts points
   (prev_xy/next_xy/back_xy: n_pairs x n_pts x 2 f32), write flags
   (bit0 fwd status, bit1 bwd status, bit2 keep; n_pairs x n_pts u8),
   kept_idx (n_pairs x n_pts) and n_kept (n_pairs). */
gvx_status gvx_klt_fb_batch_dev(gvx_ctx* ctx, int32_t n_pairs, int32_t w, int32_t h,
                                const uint8_t* d_prev, const uint8_t* d_next, int32_t n_pts,
                                const float* d_prev_xy, float* d_next_xy, float* d_back_xy,
                                uint8_t* d_flags, int32_t* d_kept_idx, int32_t* d_n_kept,
                                double fb_thresh, double border, int32_t cam_w, int32_t cam_h,
                                const gvx_klt_params* p);
/* The same with the initial flow read from d_init_xy (n_pairs x n_pts x 2 f32,
   may equal d_next_xy) and d_next_xy output only: the nextPts in / out of
   calcOpticalFlowPyrLK with OPTFLOW_USE_INITIAL_FLOW (tracking.cc:385-390) without
   a copy of the predictions into the output first. */
gvx_status gvx_klt_fb_batch_init_dev(gvx_ctx* ctx, int32_t n_pairs, int32_t w, int32_t h,
                                     const uint8_t* d_prev, const uint8_t* d_next, int32_t n_pts,
                                     const float* d_prev_xy, const float* d_init_xy, float* d_next_xy,
                                     float* d_back_xy, uint8_t* d_flags, int32_t* d_kept_idx, int32_t* d_n_kept,
                                     double fb_thresh, double border, int32_t cam_w, int32_t cam_h,
                                     const gvx_klt_params* p);
/* The batch unit in its two halves, buildOpticalFlowPyramid and
   calcOpticalFlowPyrLK on the built pyramids (the split OpenCV itself offers), so
   a caller can build batch t+1's pyramids on a gvx_branch beside batch t's LK:
   gvx_klt_batch_pyramids_dev builds levels >= 1 of the 2 * n_pairs images (prev
   images first, then next) into d_pyr (2 * n_pairs * bytes of gvx_pyramid_layout(w,
   h, max_level), image i at d_pyr + i * bytes); gvx_klt_fb_batch_pyr_dev is
   gvx_klt_fb_batch_init_dev over them.  Level 0 is read from d_prev / d_next in
   both, so those images must stay unchanged until the LK has run, and d_pyr must
   have been built from them with the same n_pairs, w, h and p->max_level.  The
   results are those of gvx_klt_fb_batch_init_dev (the same kernels). */
gvx_status gvx_klt_batch_pyramids_dev(gvx_ctx* ctx, int32_t n_pairs, int32_t w, int32_t h, const uint8_t* d_prev,
                                      const uint8_t* d_next, int32_t max_level, uint8_t* d_pyr);
gvx_status gvx_klt_fb_batch_pyr_dev(gvx_ctx* ctx, int32_t n_pairs, int32_t w, int32_t h, const uint8_t* d_prev,
                                    const uint8_t* d_next, const uint8_t* d_pyr, int32_t n_pts,
                                    const float* d_prev_xy, const float* d_init_xy, float* d_next_xy,
                                    float* d_back_xy, uint8_t* d_flags, int32_t* d_kept_idx, int32_t* d_n_kept,
                                    double fb_thresh, double border, int32_t cam_w, int32_t cam_h,
                                    const gvx_klt_params* p);
/* Host-pointer convenience wrapper of the above (copies in and out, synchronous). */
gvx_status gvx_klt_fb_batch(gvx_ctx* ctx, int32_t n_pairs, int32_t w, int32_t h,
                            const uint8_t* prev, const uint8_t* next, int32_t n_pts,
                            const float* prev_xy, float* next_xy, float* back_xy, uint8_t* flags,
                            int32_t* kept_idx, int32_t* n_kept, double fb_thresh, double border,
                            int32_t cam_w, int32_t cam_h, const gvx_klt_params* p);

/* Debug/parity hook: copy level `level` of a cached frame's pyramid (unpadded,
   w_l x h_l, tightly packed) to host.  Returns GVX_ERR_INVALID past the top. */
gvx_status gvx_frame_level(gvx_ctx* ctx, uint64_t id, int32_t level, uint8_t* out, int32_t* w,
                           int32_t* h);

/* The same level with its BORDER_REFLECT_101 border of `pad` pixels
   (0 <= pad <= GVX_PYR_PAD), (w_l + 2 pad) x (h_l + 2 pad) bytes, tightly packed:
   the padded pyramid buildOpticalFlowPyramid(..., pyrBorder = BORDER_REFLECT_101)
   hands to calcOpticalFlowPyrLK (the level plus its ring). */
#define GVX_PYR_PAD 32
gvx_status gvx_frame_level_padded(gvx_ctx* ctx, uint64_t id, int32_t level, int32_t pad, uint8_t* out);

/* Batched buildOpticalFlowPyramid (winSize 21, BORDER_REFLECT_101 pyramid border):
   the pyramids that each cv::calcOpticalFlowPyrLK call at tracking/tracking.cc:385,
   390, 487, 493 builds internally, for n_img device images (h x w u8, image i at
   d_imgs + i*img_stride, rows `stride` bytes apart) in one launch, into
   d_out + i*bytes.  gvx_pyramid_layout gives the layout: level l at byte off[l] is
   (lh[l] + 2*GVX_PYR_PAD) rows of pitch[l] bytes, the level plus its ring starting at
   its padded corner.  Levels >= 1 are always written, ring included.  Level 0 is
   read in place when w % 4 == 0 and the rows are 4-byte aligned, and its slot is then
   left unwritten; otherwise the slot holds the padded copy.  Async on the context
   stream; d_out must hold n_img * bytes. */
gvx_status gvx_pyramid_layout(int32_t w, int32_t h, int32_t max_level, int32_t* nlev, int64_t* off,
                              int32_t* pitch, int32_t* lw, int32_t* lh, int64_t* bytes);
gvx_status gvx_build_pyramids_dev(gvx_ctx* ctx, int32_t n_img, int32_t w, int32_t h, const uint8_t* d_imgs,
                                  int64_t img_stride, int32_t stride, int32_t max_level, uint8_t* d_out);

/* --------------------------------------------------------- preprocessing */
/* Tracking::preprocessing (tracking/tracking.cc:107-141): CLAHE with
   clahe_ = cv::createCLAHE(3.0, cv::Size(21, 21)) (:63) applied in place (:139),
   and the optional histogram check calculateHistigram (:88-105, used when
   track_check_histogram). */
#define GVX_CLAHE_MAX_TILES 64
typedef struct {
    double clip_limit;         /* 3.0 */
    int32_t tiles_x, tiles_y;  /* tileGridSize = (21, 21), each in [1, GVX_CLAHE_MAX_TILES] */
    int32_t channels;          /* source format: 1 = MONO8 (default), 3 = BGR8 -- converted
                                  first as cv::cvtColor(COLOR_BGR2GRAY) (tracking.cc:111-113):
                                  (B*1868 + G*9617 + R*4899 + 8192) >> 14, folded into the
                                  CLAHE histogram pass (which writes the gray frame once);
                                  strides stay in bytes (>= 3 w), the histogram check and
                                  the outputs are of the gray frame */
} gvx_clahe_params;
void gvx_clahe_params_default(gvx_clahe_params* p);

/* clahe_->apply on n images in device memory, async on the context stream.
   Image i is h x w u8 at d_src + i*src_img_stride with rows src_stride bytes
   apart (likewise d_dst); d_dst may equal d_src (in place, like the reference).
   d_hist_mean (nullable): n doubles, calculateHistigram of each SOURCE image. */
gvx_status gvx_clahe_batch_dev(gvx_ctx* ctx, int32_t n, int32_t w, int32_t h, const uint8_t* d_src,
                               int64_t src_img_stride, int32_t src_stride, uint8_t* d_dst,
                               int64_t dst_img_stride, int32_t dst_stride, const gvx_clahe_params* cp,
                               double* d_hist_mean);
/* One host image, synchronous.  hist_mean (nullable) as above. */
gvx_status gvx_clahe(gvx_ctx* ctx, int32_t w, int32_t h, const uint8_t* src, int32_t src_stride, uint8_t* dst,
                     int32_t dst_stride, const gvx_clahe_params* cp, double* hist_mean);

/* The whole per-frame preprocessing into the frame cache: calculateHistigram
   of the raw frame (when hist_mean != NULL), CLAHE, then gvx_frame_put of the
   equalised image (its pyramid).  clahe_out (nullable, w*h bytes, tightly
   packed) receives frame->image() after :139.  Synchronous. */
gvx_status gvx_frame_preprocess(gvx_ctx* ctx, uint64_t id, const uint8_t* gray, int32_t w, int32_t h,
                                int32_t stride, const gvx_clahe_params* cp, const gvx_klt_params* p,
                                double* hist_mean, uint8_t* clahe_out);
/* The same from a device image, async on the context stream; d_hist_mean and
   d_clahe_out (w*h, tightly packed) are device pointers and may be NULL. */
gvx_status gvx_frame_preprocess_dev(gvx_ctx* ctx, uint64_t id, const uint8_t* d_gray, int32_t w, int32_t h,
                                    int32_t stride, const gvx_clahe_params* cp, const gvx_klt_params* p,
                                    double* d_hist_mean, uint8_t* d_clahe_out);
/* The same for frame *d_index of a sequence resident in HBM (frame f at
   d_frames + f * frame_stride, rows `stride` bytes apart, n_frames of them), the
   index read on the device and clamped to [0, n_frames - 1]: a captured
   per-frame graph picks its frame without a host round trip (bench.py
   --config 5).  Frames of at least 66 x 66 px. */
gvx_status gvx_frame_preprocess_indexed_dev(gvx_ctx* ctx, uint64_t id, const uint8_t* d_frames,
                                            int64_t frame_stride, const int32_t* d_index, int32_t n_frames,
                                            int32_t w, int32_t h,
                                            int32_t stride, const gvx_clahe_params* cp, const gvx_klt_params* p,
                                            double* d_hist_mean);

/* ------------------------------------------------------------ camera ops */
/* Camera (tracking/camera.cc:25-46): K = [fx skew cx; 0 fy cy; 0 0 1] and the
   distortion (k1, k2, p1, p2, k3); k3 = 0 for a 4-term config (:62-64). */
typedef struct {
    double fx, fy, cx, cy, skew;
    double k1, k2, p1, p2, k3;
    int32_t width, height;
} gvx_camera;
enum {
    GVX_CAM_UNDISTORT = 0, GVX_CAM_DISTORT = 1, GVX_CAM_PREDICT = 2,
    GVX_CAM_PROJECT = 3, GVX_CAM_VELOCITY = 4, GVX_CAM_PARALLAX = 5
};

/* Per-point camera operations around the KLT calls on n points (xy: n x 2
   float pixels).  Host pointers, synchronous; each *_dev twin takes device
   pointers and is async on the context stream.  Rotations are row-major 3x3
   doubles.  Outputs may not alias inputs. */
/* Camera::undistortPoints = cv::undistortPoints(pts, pts, K, D, Mat(), K) (camera.cc:72-74) */
gvx_status gvx_undistort_points(gvx_ctx* ctx, const gvx_camera* cam, int32_t n, const float* xy, float* out);
gvx_status gvx_undistort_points_dev(gvx_ctx* ctx, const gvx_camera* cam, int32_t n, const float* d_xy, float* d_out);
/* Camera::distortPoints (camera.cc:76-89) */
gvx_status gvx_distort_points(gvx_ctx* ctx, const gvx_camera* cam, int32_t n, const float* xy, float* out);
gvx_status gvx_distort_points_dev(gvx_ctx* ctx, const gvx_camera* cam, int32_t n, const float* d_xy, float* d_out);
/* Tracking::trackReferenceFrame's initial flow (tracking.cc:465-478): undistort,
   pixel2cam, r_cur_pre * pc, distortCameraPoint (camera.cc:105-118). */
gvx_status gvx_predict_rotated(gvx_ctx* ctx, const gvx_camera* cam, const double* r_cur_pre, int32_t n,
                               const float* xy, float* out);
gvx_status gvx_predict_rotated_dev(gvx_ctx* ctx, const gvx_camera* cam, const double* r_cur_pre, int32_t n,
                                   const float* d_xy, float* d_out);
/* Tracking::trackMappoint's prediction (tracking.cc:366-377): world2pixel(pw,
   pose) (camera.cc:137-143, R/t = pose.R, pose.t) then distortPoints; pw n x 3. */
gvx_status gvx_project_points(gvx_ctx* ctx, const gvx_camera* cam, const double* R, const double* t, int32_t n,
                              const double* pw, float* out);
gvx_status gvx_project_points_dev(gvx_ctx* ctx, const gvx_camera* cam, const double* R, const double* t,
                                  int32_t n, const double* d_pw, float* d_out);
/* (pixel2cam(cur) - pixel2cam(pre)) / dt on undistorted points (tracking.cc:433,
   :530); vel n x 2 doubles. */
gvx_status gvx_point_velocity(gvx_ctx* ctx, const gvx_camera* cam, int32_t n, const float* pre, const float* cur,
                              double dt, double* vel);
gvx_status gvx_point_velocity_dev(gvx_ctx* ctx, const gvx_camera* cam, int32_t n, const float* d_pre,
                                  const float* d_cur, double dt, double* d_vel);
/* Tracking::keyPointParallax (tracking.cc:861-871) per undistorted point pair,
   R0/R1 = pose0.R / pose1.R; out n doubles (pixels). */
gvx_status gvx_keypoint_parallax(gvx_ctx* ctx, const gvx_camera* cam, const double* R0, const double* R1,
                                 int32_t n, const float* ref, const float* cur, double* out);
gvx_status gvx_keypoint_parallax_dev(gvx_ctx* ctx, const gvx_camera* cam, const double* R0, const double* R1,
                                     int32_t n, const float* d_ref, const float* d_cur, double* d_out);
/* cv::findFundamentalMat(p1, p2, FM_RANSAC, thresh, confidence, mask) with
   OpenCV's maxIters (1000 in the reference's overload), the outlier rejection
   of Tracking::trackReferenceFrame (tracking.cc:547-555: undistorted points,
   thresh = reprojection_error_std_, confidence 0.99, then reduceVector with the
   mask).  Batched over n_sets independent point sets: set i is points
   off[i] .. off[i+1] of p1 / p2 (float x, y pairs).  mask (u8 per point): 1 =
   inlier; result[i]: 1 = a model was found, 0 = none (mask all zero; OpenCV
   would leave the caller's buffer as it was), -1 = fewer than 15 points (the
   reference never calls it then: mask all one).  F (nullable): the best model
   per set, row-major 3x3. */
gvx_status gvx_find_fundamental_ransac(gvx_ctx* ctx, int32_t n_sets, const int32_t* off, const float* p1,
                                       const float* p2, double thresh, double confidence, int32_t max_iters,
                                       uint8_t* mask, double* F, int32_t* result);
gvx_status gvx_find_fundamental_ransac_dev(gvx_ctx* ctx, int32_t n_sets, const int32_t* d_off, const float* d_p1,
                                           const float* d_p2, double thresh, double confidence, int32_t max_iters,
                                           uint8_t* d_mask, double* d_F, int32_t* d_result);

/* ------------------------------------------------------ feature detection */
/* Tracking::featuresDetection (tracking/tracking.cc:576-688): block grid from
   the Tracking ctor (:65-85), FILLED circle mask of radius
   track_min_pixel_distance_ (:609-620), per block goodFeaturesToTrack
   (quality 0.01, blockSize 3) + cornerSubPix(5x5, 20 it, 0.01) (:647-651). */
typedef struct {
    double block_size;   /* TRACK_BLOCK_SIZE = 200 */
    int32_t max_features;/* track_max_features */
    double quality;      /* 0.01 */
    int32_t subpix_win;  /* 5 */
    int32_t subpix_iters;/* 20 */
    double subpix_eps;   /* 0.01 */
} gvx_detect_params;
void gvx_detect_params_default(gvx_detect_params* p);

/* count_xy: key points counted per block (frame->features() + pts2d_new_);
   mask_xy: circle centres (frame_cur_->features() + pts2d_new_); ismask as in
   the reference; n_existing = features + pts2d_ref_ for the early exit
   (*n_out = -1 when it triggers).  out_xy holds up to block_cnts *
   max_block_features points, block-major like the reference's merge loop;
   out_block_counts has block_cnts entries. */
gvx_status gvx_detect(gvx_ctx* ctx, uint64_t frame_id, const float* count_xy, int32_t n_count,
                      const float* mask_xy, int32_t n_mask, int32_t ismask, int32_t n_existing,
                      const gvx_detect_params* p, float* out_xy, int32_t* out_block_counts,
                      int32_t* n_out);

/* ------------------------------------------- one frame, device-resident */
/* Tracking::track's image path for one frame (tracking/tracking.cc:144-245, the
   parts SequenceTracker follows) with the tracker state in device memory and no
   host round trip: when `track`, forward + backward LK of the *d_n points d_pts
   from prev_frame into next_frame with the initial flow d_init, the FB / border /
   status filter and reduceVector (:380-408, :831-849), giving d_pts <- tracked,
   d_vel <- tracked - previous, d_init <- d_pts + d_vel, *d_n <- kept; then, while
   *d_n < max_features (and not above max_features - 5), featuresDetection on
   next_frame (:576-688) with the tracked points as counts and mask, its corners
   appended in block order up to max_features (vel 0).  capacity >= max_features
   entries per state array.  d_kept (nullable): the kept indices; d_corners
   (nullable, blocks x maxCorners float2) / d_n_corners: every detected corner and
   their count (-1: detection skipped).  Every count stays on the device, so after
   one uncaptured call (it uploads the detection constants) the call can be
   captured into a hipGraph and replayed per frame. */
gvx_status gvx_track_frame_dev(gvx_ctx* ctx, uint64_t prev_frame, uint64_t next_frame, int32_t track, float* d_pts,
                               float* d_vel, float* d_init, int32_t* d_n, int32_t capacity, int32_t cam_w,
                               int32_t cam_h, double fb_thresh, double border, const gvx_klt_params* klt,
                               const gvx_detect_params* detect, int32_t* d_kept, float* d_corners,
                               int32_t* d_n_corners);
/* The part of featuresDetection that depends on the frame alone -- the
   cornerMinEigenVal map of every detection block (goodFeaturesToTrack's
   eigenvalue image, tracking.cc:647) -- computed for frame `frame` now, on the
   context stream, and kept with the frame until it is written again.  A later
   gvx_track_frame_[record_]dev on that frame with the same detection grid then
   reads it instead of launching it, so a pipelined tracker can put it on the
   branch that prepares the next frame (off the tracking critical path).
   Replaces: nothing in the reference (an evaluation-order split of :647). */
gvx_status gvx_frame_eig_dev(gvx_ctx* ctx, uint64_t frame, const gvx_detect_params* detect);
/* gvx_track_frame_dev followed by gvx_track_record_dev (below) on the same state,
   the record appended by the detection's last kernel (one launch less per frame). */
gvx_status gvx_track_frame_record_dev(gvx_ctx* ctx, uint64_t prev_frame, uint64_t next_frame, int32_t track,
                                      float* d_pts, float* d_vel, float* d_init, int32_t* d_n, int32_t capacity,
                                      int32_t cam_w, int32_t cam_h, double fb_thresh, double border,
                                      const gvx_klt_params* klt, const gvx_detect_params* detect, float* d_tracks,
                                      int32_t* d_counts, int32_t* d_frame_index, int32_t max_frames);
/* Helpers that keep a replay loop inside one captured graph per frame: copy
   bytes from d_src_base + (*d_index) * bytes (e.g. frame *d_index of a sequence
   resident in HBM; the index clamped to [0, n_src - 1]), and append the current track list (*d_n points of d_pts) to
   d_tracks[*d_frame_index * capacity ..] / d_counts[*d_frame_index], then
   advance *d_frame_index (frames >= max_frames are not stored). */
gvx_status gvx_copy_indexed_dev(gvx_ctx* ctx, void* d_dst, const void* d_src_base, size_t bytes,
                                const int32_t* d_index, int32_t n_src);
gvx_status gvx_track_record_dev(gvx_ctx* ctx, const float* d_pts, const int32_t* d_n, int32_t capacity,
                                float* d_tracks, int32_t* d_counts, int32_t* d_frame_index, int32_t max_frames);
/* *d_index += delta on the context stream (a frame counter that a captured
   graph advances for itself, e.g. the pipelined replay's preprocessing branch). */
gvx_status gvx_index_advance_dev(gvx_ctx* ctx, int32_t* d_index, int32_t delta);


/* --------------------------------------------------- IMU preintegration */
enum { GVX_PREINT_NORMAL = 0, GVX_PREINT_EARTH = 2 }; /* preintegration.h:38-43 */

/* IMU record, common/types.h:50-58. */
typedef struct {
    double time, dt, dtheta[3], dvel[3], odovel;
} gvx_imu;

/* IntegrationParameters subset on the path (preintegration/integration_state.h:68-89). */
typedef struct {
    double acc_vrw, gyr_arw, gyr_bias_std, acc_bias_std, corr_time, gravity;
} gvx_imu_params;

/* IntegrationState core (integration_state.h:35-51); q = (x, y, z, w). */
typedef struct {
    double time;
    double p[3], q[4], v[3], bg[3], ba[3];
} gvx_state;

/* A PreintegrationBase after its segment: deltaState(), currentState(),
   deltaTime(), jacobian_, covariance_ (row-major 15x15), plus what the Earth
   variant's evaluate() needs (iewn_, gravity_).  sqrt_info is
   sqrt_information_ = LLT(covariance_^-1).matrixL().transpose() (row-major,
   upper triangular): the reference recomputes it inside every
   PreintegrationFactor::Evaluate (preintegration_earth.cc:39-40,
   preintegration_normal.cc), but it depends on covariance_ alone, so
   gvx_preint_integrate[_dev] forms it once per segment with the same
   arithmetic (identical bits) and the factor kernels read it.  A result built
   by other means must pass through gvx_preint_sqrt_info[_dev] first. */
typedef struct {
    int32_t variant, m; /* m = imu_buffer_.size() */
    double delta_time, start_time, end_time;
    gvx_state current, delta;
    double gravity[3], iewn[3], q0[4];
    double jacobian[225];
    double covariance[225];
    double sqrt_info[225];
} gvx_preint_result;

/* (Re)compute pre[i].sqrt_info from pre[i].covariance for n results in place
   (partial-pivot LU inverse, then Eigen's unblocked LLT; one wavefront per
   result).  Called by gvx_preint_integrate[_dev] and gvx_factor_set_create. */
gvx_status gvx_preint_sqrt_info(gvx_ctx* ctx, int32_t n, gvx_preint_result* pre);
gvx_status gvx_preint_sqrt_info_dev(gvx_ctx* ctx, int32_t n, gvx_preint_result* d_pre);

/* Preintegration::createPreintegration + addNewImu(series[k]), k = 1..m-1
   (ic_gvins.cc:946-953, preintegration_base.cc:72-75), batched over segments:
   segment s uses imu[seg_off[s] .. seg_off[s+1]) and state0[s]; iewn[s] is the
   Earth rate computed by the caller as PreintegrationEarth::resetState does
   (gvx_earth_iewn); ignored for NORMAL.  pn (Earth only, may be NULL) receives
   the pn_ list {dt, p[3]} per integrated step: (seg_off[s]-s) * 4 doubles
   offset for segment s.  One wavefront per segment. */
gvx_status gvx_preint_integrate(gvx_ctx* ctx, int32_t variant, const gvx_imu_params* prm,
                                int32_t n_seg, const gvx_imu* imu, const int32_t* seg_off,
                                const gvx_state* state0, const double* iewn,
                                gvx_preint_result* out, double* pn);
gvx_status gvx_preint_integrate_dev(gvx_ctx* ctx, int32_t variant, const gvx_imu_params* prm,
                                    int32_t n_seg, const gvx_imu* d_imu, const int32_t* d_seg_off,
                                    const gvx_state* d_state0, const double* d_iewn,
                                    gvx_preint_result* d_out, double* d_pn);
/* Which form gvx_preint_integrate[_dev] runs (default GVX_PREINT_PATH_AUTO:
   the two-launch form -- preint_pre_kernel forms the per-step terms and runs
   the quaternion chains as wave prefix products, then preint_cov16_kernel runs
   the covariance pass with sqrt_information_ in its epilogue -- whenever its
   scratch can be sized; the single kernel otherwise).  GVX_PREINT_PATH_ONEPHASE forces the
   single kernel: an A/B and parity switch, per context.  The environment
   variable GVX_PREINT_ONEPHASE=1 sets it when the context is created. */
#define GVX_PREINT_PATH_AUTO 0
#define GVX_PREINT_PATH_ONEPHASE 1
gvx_status gvx_set_preint_path(gvx_ctx* ctx, int32_t path);

/* How the batched LK launches (more than 4,096 points, the exact window-sum
   order: three points per wave) are cut (tracking.cc:385-408, the calls they
   replace): `levels_per_phase` >= 1 runs every point group's chain -- forward
   levels maxLevel..0, then backward -- as phases of that many levels, one wave
   each, handing the flow on through device memory (DESIGN 4 "LK phases");
   0 (default) runs each group's whole chain in one wave.  The groups are
   dispatched in superchunks of `groups_per_chunk` (rounded down to a multiple
   of 8; 0 keeps the current value, default 4096), each superchunk phase by
   phase.  Same bits either way.  The environment variables GVX_KLT_LPP and
   GVX_KLT_SUPER set them when the context is created. */
gvx_status gvx_set_klt_phases(gvx_ctx* ctx, int32_t levels_per_phase, int32_t groups_per_chunk);

/* Earth::iewn(station, p) (common/earth.h:233-237), host-side helper used by
   resetState (preintegration_earth.cc:320). */
void gvx_earth_iewn(const double origin[3], const double local[3], double iewn[3]);

/* ------------------------------------------------ remaining window factors */
/* The other cost functions of the sliding window (ic_gvins.cc:1193, :1959-1990),
   batched: factor i reads its parameter block at params + offs[i] (params holds
   n_params doubles) and its constants at consts + i * NC; R residuals and an
   R x P row-major Jacobian (like Ceres) per factor, jacobians may be NULL.
     GVX_FACTOR_GNSS        GnssFactor::Evaluate (factors/gnss_factor.h:52-95):
                            pose[7]; consts {blh[3], std[3], lever[3]}; R 3, P 7, NC 9
     GVX_FACTOR_IMU_ERROR   ImuErrorFactor::Evaluate, NORMAL / EARTH options
                            (preintegration/imu_error_factor.h:45-66): mix[9]; R 6, P 9, NC 0
     GVX_FACTOR_POSE_PRIOR  ImuPosePriorFactor::Evaluate (imu_pose_prior_factor.h:42-68):
                            pose[7]; consts {prior pose[7], std[6]}; R 6, P 7, NC 13
     GVX_FACTOR_MIX_PRIOR   ImuMixPriorFactor::Evaluate, NORMAL / EARTH options
                            (imu_mix_prior_factor.h:40-56): mix[9]; consts {prior mix[9],
                            std[9]}; R 9, P 9, NC 18 */
enum { GVX_FACTOR_GNSS = 0, GVX_FACTOR_IMU_ERROR = 1, GVX_FACTOR_POSE_PRIOR = 2, GVX_FACTOR_MIX_PRIOR = 3 };
gvx_status gvx_small_factor_eval(gvx_ctx* ctx, int32_t kind, int32_t n, const double* consts, const double* params,
                                 int32_t n_params, const int32_t* offs, double* residuals, double* jacobians);
gvx_status gvx_small_factor_eval_dev(gvx_ctx* ctx, int32_t kind, int32_t n, const double* d_consts,
                                     const double* d_params, const int32_t* d_offs, double* d_residuals,
                                     double* d_jacobians);

/* MarginalizationFactor::Evaluate (factors/marginalization_factor.h:54-110),
   r = remainedSize() (<= 8192).  Remained block b: size[b] (7 = pose, local
   size 6), index[b] = remainedBlockIndex()[b] - marginalizedSize(), values at
   params + xoff[b] (current; n_x doubles in all) and x0 + xoff[b]
   (remainedBlockData(), the linearisation point).  J0 = linearizedJacobians()
   (r x r, column-major as Eigen stores it), e0 = linearizedResiduals().
   residuals r; jacobians (may be NULL): block b at jacobians + r * xoff[b],
   row-major r x size[b]. */
gvx_status gvx_marg_factor_eval(gvx_ctx* ctx, int32_t r, int32_t nb, const int32_t* size, const int32_t* index,
                                const int32_t* xoff, int32_t n_x, const double* x0, const double* params,
                                const double* J0, const double* e0, double* residuals, double* jacobians);

/* ------------------------------------------------------- marginalisation */
/* MarginalizationInfo::marginalization() once its residual blocks are evaluated
   (factors/marginalization_info.h:73-101): constructEquation (:195-230,
   H0 = sum J^T J, b0 = -sum J^T e over the local columns), schurElimination
   (:170-192, Hmm^-1 through Eigen's SelfAdjointEigenSolver with eigenvalues
   <= 1e-8 dropped, Hp = Hrr - Hrm Hmm^-1 Hmr, bp = brr - Hrm Hmm^-1 bm) and
   linearization (:153-167, J0 = S^1/2 V^T, e0 = -S^-1/2 V^T bp of Hp's
   eigen-decomposition), all on the device.
   Residual block f (ResidualBlockInfo, factors/residual_block_info.h): nres[f]
   residuals at data[res_off[f]]; its parameter blocks are blk[blk_off[f] ..
   blk_off[f+1]) (ids into the block table), and their row-major nres x size
   Jacobians follow one another from data[jac_off[f]] (ResidualBlockInfo::
   jacobians(), Ceres' global columns).  loss (nullable): per-block HuberLoss
   parameter, <= 0 for none (the reference passes nullptr, ic_gvins.cc:1529-1642;
   ResidualBlockInfo::Evaluate :59-87 corrects by sqrt(rho')).
   Block table: size[b] = global size (7 = pose, local 6), index[b] = local
   offset in H0 as updateParameterBlocksIndex (:232-253) assigns it (marginalized
   blocks first); m = marginalizedSize() > 0, L = local size, r = L - m; m and r
   at most 512.  Outputs: J0 (r x r column-major, linearizedJacobians()), e0 [r]
   (linearizedResiduals()); optional Hp (r x r column-major), bp [r], eval [r]
   (Hp's eigenvalues, ascending; NaN where the FAST solver's Cholesky path ran,
   gvx_set_marg_solver below) and info [2] (the two eigen solves: 0 = Success,
   1 = NoConvergence, which the reference does not check either). */
gvx_status gvx_marginalize(gvx_ctx* ctx, int32_t n_fac, const int32_t* nres, const int32_t* blk_off,
                           const int32_t* blk, const int64_t* res_off, const int64_t* jac_off, const double* data,
                           int64_t n_data, const double* loss, int32_t nb, const int32_t* size, const int32_t* index,
                           int32_t m, int32_t L, double* J0, double* e0, double* Hp, double* bp, double* eval,
                           int32_t* info);
/* The solver of schurElimination / linearization (per context, default FAST):
   EXACT  Eigen's SelfAdjointEigenSolver for both Hmm^-1 and Hp's factor, bit-exact
          against the restatement (oracle/marg.c) -- the reference's arithmetic;
   FAST   where Hmm - 1e-8*I (resp. Hp - 1e-8*I) is positive definite, i.e. no
          eigenvalue is dropped, Cholesky factors instead: Hp = Hrr - X^T X with
          X = Lm^-1 Hmr, J0 = Lp^T, e0 = -Lp^-1 bp.  Hp and bp are the same matrix
          and vector (to rounding; Hmm's conditioning bounds the difference), and
          J0^T J0 = Hp, J0^T e0 = -bp as in the reference, so the marginalisation
          prior ||e0 + J0 dx||^2 is the same function; J0 / e0 themselves differ
          by an orthogonal transform, and eval is NaN.  Where the check fails
          (an eigenvalue <= 1e-8) that step runs the EXACT solver.  The check is
          decided on the device (no host round trip). */
#define GVX_MARG_SOLVER_EXACT 0
#define GVX_MARG_SOLVER_FAST 1
gvx_status gvx_set_marg_solver(gvx_ctx* ctx, int32_t solver);
/* The same with data, loss and every output as device pointers (d_info: 2 ints,
   nullable), enqueued on the context stream; the structure arrays stay host
   arrays (the host turns them into the per-pair contribution lists).  Waits
   for earlier work on the stream before it reuses its pinned list staging. */
gvx_status gvx_marginalize_dev(gvx_ctx* ctx, int32_t n_fac, const int32_t* nres, const int32_t* blk_off,
                               const int32_t* blk, const int64_t* res_off, const int64_t* jac_off,
                               const double* d_data, int64_t n_data, const double* d_loss, int32_t nb,
                               const int32_t* size, const int32_t* index, int32_t m, int32_t L, double* d_J0,
                               double* d_e0, double* d_Hp, double* d_bp, double* d_eval, int32_t* d_info);
/* ------------------------------------------- LM step: DENSE_SCHUR reduced system */
/* One Levenberg-Marquardt linear step of the sliding-window BA as Ceres takes
   it with linear_solver_type = DENSE_SCHUR (ic_gvins.cc:1170-1180; Solve at
   :1217 and :1251): the normal equations of the evaluated residual blocks,
   (J^T J + diag(D^2)) delta = -J^T r, with the e-blocks (the landmarks' inverse
   depths: local indices [0, m)) eliminated --
     S = Hff - Hfe Hee^-1 Hef       (the reduced camera system, dense),
     S delta_f = bf - Hfe Hee^-1 be  by Cholesky,
     delta_e = Hee^-1 (be - Hef delta_f),     with b = -J^T r.
   Residual blocks and block table as gvx_marginalize (pose blocks of global size
   7 contribute their local 6 columns, PoseParameterization's [I6; 0]); L - m
   at most 512, and m at most 512 unless Hee is diagonal -- every eliminated
   block of local size 1 and no factor coupling two of them, the reference's
   window of one inverse depth per landmark -- which any m may have (Hee's
   Cholesky factor is then its square root); J and r are what Ceres' linear solver sees (robust-loss
   corrections applied).  D (nullable, L local parameters): the LM
   regularisation.  Outputs: delta [L] in local index order; S (nullable, r x r
   column-major, r = L - m) and info (nullable, 2 ints: 1 where the Cholesky
   factorisation of Hee + D, resp. S, met a non-positive pivot, else 0; a
   failed Hee + D also sets info[1], since S is then never formed).  When either
   factorisation fails every entry of delta is NaN and gvx_schur_solve returns
   GVX_ERR_NUMERIC after writing delta, S and info (Ceres' linear solver
   reports FAILURE and LM rejects the step).  The window holds at most
   GVX_SCHUR_MAX_L local parameters (L; the dense H0 is L x L fp64, 2 GiB at the
   bound): larger ones return GVX_ERR_UNSUPPORTED. */
#define GVX_SCHUR_MAX_L 16384
gvx_status gvx_schur_solve(gvx_ctx* ctx, int32_t n_fac, const int32_t* nres, const int32_t* blk_off,
                           const int32_t* blk, const int64_t* res_off, const int64_t* jac_off, const double* data,
                           int64_t n_data, int32_t nb, const int32_t* size, const int32_t* index, int32_t m,
                           int32_t L, const double* D, double* delta, double* S, int32_t* info);
/* The same with data, D and the outputs as device pointers, enqueued on the
   context stream (the structure arrays stay host arrays).  Asynchronous: a
   failed factorisation shows as NaN in d_delta and in d_info only. */
gvx_status gvx_schur_solve_dev(gvx_ctx* ctx, int32_t n_fac, const int32_t* nres, const int32_t* blk_off,
                               const int32_t* blk, const int64_t* res_off, const int64_t* jac_off,
                               const double* d_data, int64_t n_data, int32_t nb, const int32_t* size,
                               const int32_t* index, int32_t m, int32_t L, const double* d_D, double* d_delta,
                               double* d_S, int32_t* d_info);

/* Eigen::SelfAdjointEigenSolver<MatrixXd>(A) with eigenvectors, the solver both
   steps above use: A n x n column-major (ld lda), lower triangle read, n <= 512.
   w [n] ascending, V n x n column-major, info 0 / 1 (NoConvergence). */
gvx_status gvx_sym_eigen(gvx_ctx* ctx, int32_t n, const double* A, int32_t lda, double* w, double* V,
                         int32_t* info);

/* ------------------------------------------------------ INS mechanization */
/* IntegrationConfiguration as MISC::insMechanization reads it
   (integration_state.h:91-99): iswithearth selects the Earth-rotation variant
   (Coriolis term, qnn = q(-iewn dt)); gravity is the navigation-frame vector. */
typedef struct {
    int32_t iswithearth;
    double gravity[3];
    double iewn[3];
} gvx_ins_config;

/* The chain insMechanization(imu[k-1], imu[k], state), k = 1 .. m-1
   (misc.cc:174-229; the loop of redoInsMechanization misc.cc:269-275 and the
   per-sample call of ic_gvins.cc:304-310), batched over chains: chain i uses
   imu[off[i] .. off[i+1]) and starts from state0[i]; states[off[i]] = state0[i]
   and states[off[i]+k] is the state after sample k.  One wavefront per chain. */
gvx_status gvx_ins_propagate(gvx_ctx* ctx, const gvx_ins_config* cfg, int32_t n_chain, const gvx_imu* imu,
                             const int32_t* off, const gvx_state* state0, gvx_state* states);
gvx_status gvx_ins_propagate_dev(gvx_ctx* ctx, const gvx_ins_config* cfg, int32_t n_chain, const gvx_imu* d_imu,
                                 const int32_t* d_off, const gvx_state* d_state0, gvx_state* d_states);

/* MISC::redoInsMechanization (misc.cc:231-284) on a window of n samples and
   their states, updated in place from the sample after updated->time on (the
   caller trims the window, as the reference's pop_front does).  *index =
   getInsWindowIndex (0: updated->time outside the window, nothing changes). */
gvx_status gvx_redo_ins_mechanization(gvx_ctx* ctx, const gvx_ins_config* cfg, const gvx_state* updated,
                                      int32_t n, const gvx_imu* imu, gvx_state* states, int32_t* index);

/* MISC::getImuSeriesFromTo (misc.cc:330-384), host logic (no device): the IMU
   series over [start, end] with the boundary samples split; series must hold
   n + 2 records.  GVX_ERR_NOT_FOUND when start or end is outside the window. */
gvx_status gvx_imu_series_from_to(const gvx_imu* imu, int32_t n, double start, double end, gvx_imu* series,
                                  int32_t* n_series);

/* ------------------------------------------------------ factor batches */
/* PreintegrationFactor::Evaluate (preintegration/preintegration_factor.h:45-69)
   for n factors: factor i uses pre[i], pn list at pn[pn_off[i]*4 ...]
   (pre[i].m - 1 entries of 4 doubles; n_pn entries in total, Earth only --
   pn/pn_off may be NULL when every factor is NORMAL), and parameter blocks
   params + offs[4i+k] (params holds n_params doubles) (k:
   pose0[7], mix0[9], pose1[7], mix1[9]).  residuals n x 15; jacobians (may be
   NULL) n x 480 doubles = [J_pose0 15x7 | J_mix0 15x9 | J_pose1 15x7 |
   J_mix1 15x9], each row-major like Ceres.  pre[i].sqrt_info must be filled
   (gvx_preint_integrate does; otherwise gvx_preint_sqrt_info): the host entry
   refuses a result whose sqrt_info diagonal is not positive. */
gvx_status gvx_preint_factor_eval(gvx_ctx* ctx, int32_t n, const gvx_preint_result* pre,
                                  const double* pn, int32_t n_pn, const int32_t* pn_off,
                                  const double* params, int32_t n_params, const int32_t* offs,
                                  double* residuals, double* jacobians);
gvx_status gvx_preint_factor_eval_dev(gvx_ctx* ctx, int32_t n, const gvx_preint_result* d_pre,
                                      const double* d_pn, const int32_t* d_pn_off,
                                      const double* d_params, const int32_t* d_offs,
                                      double* d_residuals, double* d_jacobians);

/* ReprojectionFactor constants (factors/reprojection_factor.h:47-58). */
typedef struct {
    double pts0[3], pts1[3], vel0[3], vel1[3], td0, td1, std;
} gvx_reproj_const;

/* ReprojectionFactor::Evaluate (factors/reprojection_factor.h:61-161) for n
   factors; factor i reads params + offs[5i+k] (pose_ref[7], pose_obs[7],
   ext[7], invdepth[1], td[1]).  residuals n x 2; jacobians (may be NULL)
   n x 46 doubles = [J0 2x7 | J1 2x7 | J2 2x7 | J3 2x1 | J4 2x1]. */
gvx_status gvx_reproj_eval(gvx_ctx* ctx, int32_t n, const gvx_reproj_const* c,
                           const double* params, int32_t n_params, const int32_t* offs,
                           double* residuals, double* jacobians);
gvx_status gvx_reproj_eval_dev(gvx_ctx* ctx, int32_t n, const gvx_reproj_const* d_c,
                               const double* d_params, const int32_t* d_offs,
                               double* d_residuals, double* d_jacobians);
/* gvx_reproj_eval_dev then gvx_preint_factor_eval_dev over one parameter array
   in one call (a window's two factor kinds, what gvx_factors_prepare evaluates),
   async on the context stream.  Either count may be 0. */
gvx_status gvx_factor_batch_eval_dev(gvx_ctx* ctx, int32_t n_reproj, const gvx_reproj_const* d_rc,
                                     const int32_t* d_roffs, double* d_rres, double* d_rjac, int32_t n_preint,
                                     const gvx_preint_result* d_pre, const double* d_pn, const int32_t* d_pn_off,
                                     const int32_t* d_poffs, double* d_pres, double* d_pjac,
                                     const double* d_params);

/* ------------------------------------------- two-phase factor evaluation */
/* The Ceres EvaluationCallback pattern: a factor set holds one
   sliding window's factors; gvx_factors_prepare (called from
   ceres::EvaluationCallback::PrepareForEvaluation, after Ceres has written the
   candidate point into the user's parameter blocks) gathers the parameter
   blocks, evaluates every factor's residuals (and Jacobians) in one pass on the
   device and keeps the results in host memory owned by the set; each
   CostFunction::Evaluate then copies its slice with gvx_factor_read_*.

   Parameter blocks are host arrays registered once: blocks[b] points at
   block_sizes[b] doubles (the user's state / landmark storage, read at every
   prepare).  Reprojection factor i uses blocks r_blocks[5i+k] (pose_ref 7,
   pose_obs 7, ext 7, invdepth 1, td 1); preintegration factor i uses pre[i],
   its pn list at pn[4*pn_off[i]] (Earth) and blocks p_blocks[4i+k] (pose0 7,
   mix0 9, pose1 7, mix1 9).  The set keeps copies of the constants. */
typedef struct gvx_factor_set gvx_factor_set;

gvx_status gvx_factor_set_create(gvx_ctx* ctx, int32_t n_blocks, const double* const* blocks,
                                 const int32_t* block_sizes, int32_t n_reproj, const gvx_reproj_const* rc,
                                 const int32_t* r_blocks, int32_t n_preint, const gvx_preint_result* pre,
                                 const double* pn, int32_t n_pn, const int32_t* pn_off,
                                 const int32_t* p_blocks, gvx_factor_set** out);
void gvx_factor_set_destroy(gvx_factor_set* set);

/* Phase 1: evaluate every factor at the current block values (with_jacobians
   0: residuals only).  Synchronous; not to be overlapped with reads. */
gvx_status gvx_factors_prepare(gvx_factor_set* set, int32_t with_jacobians);

/* Phase 2: factor i's residuals and Jacobian blocks in the Ceres layout
   (row-major num_residuals x block_size); jacobians and any jacobians[k] may
   be NULL.  Reads only the set's host buffers: reentrant and lock-free, safe
   from concurrent Ceres worker threads.  GVX_ERR_INVALID if Jacobians are asked
   for after a residual-only prepare, or for an index out of range. */
gvx_status gvx_factor_read_reproj(const gvx_factor_set* set, int32_t i, double* residuals, double** jacobians);
gvx_status gvx_factor_read_preint(const gvx_factor_set* set, int32_t i, double* residuals, double** jacobians);

#ifdef __cplusplus
}
#endif

#endif /* GVX_H */
