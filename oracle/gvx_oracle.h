/*
 * gvx_oracle.h -- CPU restatement of the IC-GVINS per-frame hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libgvx.so, the C ABI in
 * include/gvx.h, the host mirror under ic-gvins_amd/) links, loads or calls
 * this code.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg use it -- as the parity checker and as the timed CPU baseline.
 *
 * PARITY STATUS: the reference (WZXTP/IC-GVINS) cannot be built or imported in
 * this environment (OpenCV, Eigen, Ceres absent -- SURVEY.md section 8c) and it
 * ships no tests, golden vectors or fixtures for this path.  This restatement is
 * therefore "parity unpinned" with respect to the real reference binaries.  It is
 * pinned instead by analytic known-answer tests (integer-shift image pairs,
 * constant/ramp pyramids, zero-rotation IMU segments, numeric-derivative checks
 * of every factor Jacobian) in tests/test_oracle_*.py.
 *
 * What each function restates (file:line in /root/reference, or the un-vendored
 * OpenCV 4.x routine the reference calls there):
 *   orc_build_pyramid      cv::buildOpticalFlowPyramid + pyrDown, called inside
 *                          cv::calcOpticalFlowPyrLK at
 *                          ic_gvins/ic_gvins/tracking/tracking.cc:385,390,487,493
 *   orc_scharr             calcSharrDeriv (same call sites)
 *   orc_calc_optical_flow_pyr_lk   cv::calcOpticalFlowPyrLK / LKTrackerInvoker
 *   orc_klt_fb             tracking.cc:383-408 (fwd + bwd LK, FB/border status,
 *                          reduceVector tracking.cc:831-849)
 *   orc_features_detection tracking.cc:576-688 (block grid, circle mask,
 *                          goodFeaturesToTrack + cornerSubPix per block)
 *   orc_preint_*           preintegration/preintegration_{base,earth,normal}.cc
 *   orc_preint_factor_eval preintegration/preintegration_factor.h:45-69
 *   orc_reproj_eval        factors/reprojection_factor.h:61-161
 *   orc_undistort_points .. orc_keypoint_parallax  per-point camera operations
 *                          around the KLT calls (camera.c; tracking/camera.cc:72-143,
 *                          tracking.cc:366-377, :419-437, :462-478, :514-544, :861-871)
 *   orc_ins_* / orc_imu_series_from_to  INS mechanization and IMU-series
 *                          extraction (ins.c; misc.cc:40-83, :174-384)
 *   orc_small_factor_eval / orc_marg_factor_eval  GNSS, ImuError, pose / mix
 *                          prior and marginalisation factors (aux_factors.c;
 *                          factors/gnss_factor.h:52-95, preintegration/
 *                          imu_error_factor.h:45-66, imu_pose_prior_factor.h:42-68,
 *                          imu_mix_prior_factor.h:40-56, factors/marginalization_factor.h:54-110)
 *   orc_clahe / orc_hist_mean  Tracking::preprocessing (tracking.cc:107-141):
 *                          cv::createCLAHE(3.0, Size(21,21))->apply and
 *                          calculateHistigram (clahe.c)
 *
 * Documented choices where the upstream arithmetic is build-dependent:
 *   - LK window sums (A11/A12/A22, b1/b2) are exact int64 sums converted to
 *     float once (OpenCV's x86 SIMD path accumulates float partials in 4-lane
 *     groups; the result differs by float rounding only).
 *   - All float/double expressions are evaluated left-to-right with no FMA
 *     contraction (-ffp-contract=off), following OpenCV's scalar tail loops and
 *     Eigen's coefficient-wise expression order.
 */
#ifndef GVX_ORACLE_H
#define GVX_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------- */
/* KLT (pyramidal Lucas-Kanade)                                               */
/* ------------------------------------------------------------------------- */

#define ORC_MAX_LEVELS 8

typedef struct {
    int win;            /* window side, 21 in the reference (tracking.cc:386) */
    int max_level;      /* TRACK_PYRAMID_LEVEL = 3 (tracking.h:113) */
    int max_iter;       /* TermCriteria COUNT = 30 */
    double eps;         /* TermCriteria EPS = 0.01 (squared internally) */
    int use_initial_flow; /* OPTFLOW_USE_INITIAL_FLOW */
    float min_eig;      /* minEigThreshold default 1e-4 */
} orc_klt_params;

/* A padded u8 plane: pixel (x, y) lives at buf[(y + pad) * pitch + x + pad]. */
typedef struct {
    int w, h, pad, pitch;
    uint8_t* buf;
} orc_u8plane;

/* A padded interleaved int16 (dx, dy) plane. */
typedef struct {
    int w, h, pad, pitch; /* pitch in (dx,dy) pairs */
    int16_t* buf;
} orc_s16plane;

typedef struct {
    int nlevels;
    orc_u8plane lv[ORC_MAX_LEVELS];
} orc_pyramid;

void orc_klt_params_default(orc_klt_params* p);
/* Window-sum accumulation order of LK (klt.c; parity experiment). */
enum { ORC_ACC_EXACT = 0, ORC_ACC_F32 = 1, ORC_ACC_F32X4 = 2 };
void orc_set_lk_accum(int mode);

/* Returns the highest level built (<= max_level). Levels are padded by `win`
   pixels with BORDER_REFLECT_101, exactly as buildOpticalFlowPyramid does. */
int orc_build_pyramid(const uint8_t* img, int w, int h, int stride, int win, int max_level,
                      orc_pyramid* pyr);
void orc_free_pyramid(orc_pyramid* pyr);

/* Scharr derivative of an unpadded view (x in [0,w), y in [0,h)) of `src`,
   written interleaved (dx, dy) into out[(y*w + x)*2 + {0,1}]. */
void orc_scharr(const orc_u8plane* src, int16_t* out);

/* Exact restatement of cv::calcOpticalFlowPyrLK(prev, next, prevPts, nextPts,
   status, err, Size(win,win), max_level, TermCriteria(COUNT+EPS, iters, eps),
   flags, minEig) on u8 gray images.  nextPts is in/out when use_initial_flow.
   Builds both pyramids itself (as OpenCV does on every call).  nthreads > 1
   splits the point range like OpenCV's parallel_for_. */
void orc_calc_optical_flow_pyr_lk(const uint8_t* prev, const uint8_t* next, int w, int h, int stride,
                                  const float* prev_xy, float* next_xy, uint8_t* status, float* err,
                                  int n, const orc_klt_params* p, int nthreads);

/* Same, on pyramids built by the caller (pyramid-reuse variant). */
void orc_lk_on_pyramids(const orc_pyramid* prev, const orc_pyramid* next, const float* prev_xy,
                        float* next_xy, uint8_t* status, float* err, int n, const orc_klt_params* p,
                        int nthreads);

/* tracking.cc:383-408: forward LK, backward LK (initial flow = prev points),
   keep = st_f && st_b && !isOnBorder(next) && ptsDistance(back, prev) < fb_thresh,
   then order-preserving compaction.  `border` is the isOnBorder margin (5.0),
   cam_w/cam_h the camera size used by isOnBorder.
   Outputs: next_xy (in: initial flow, out: forward result), back_xy, st_f, st_b,
   keep[n], kept_idx[*n_kept].  Returns n_kept.
   reuse_pyramids = 0 follows the reference's call pattern (each LK call builds
   both pyramids again); 1 builds each pyramid once. */
int orc_klt_fb(const uint8_t* prev, const uint8_t* next, int w, int h, int stride,
               const float* prev_xy, float* next_xy, float* back_xy, uint8_t* st_f, uint8_t* st_b,
               uint8_t* keep, int* kept_idx, int n, double fb_thresh, double border, int cam_w,
               int cam_h, const orc_klt_params* p, int reuse_pyramids, int nthreads);

/* ------------------------------------------------------------------------- */
/* Feature detection (block-grid GFTT + cornerSubPix)                         */
/* ------------------------------------------------------------------------- */

typedef struct {
    double block_size;      /* TRACK_BLOCK_SIZE = 200 (tracking.h:112) */
    int max_features;       /* track_max_features (config) */
    double quality;         /* 0.01 (tracking.cc:647) */
    int subpix_win;         /* 5 (tracking.cc:623) */
    int subpix_iters;       /* 20 */
    double subpix_eps;      /* 0.01 */
} orc_detect_params;

typedef struct {
    int block_cols, block_rows, block_cnts;
    int col, row;           /* block_indexs_[0] = (col, row) */
    int max_block_features; /* track_max_block_features_ */
    int min_pixel_distance; /* track_min_pixel_distance_ */
} orc_block_grid;

void orc_detect_params_default(orc_detect_params* p);
/* Tracking ctor, tracking.cc:65-85. */
void orc_block_grid_make(int w, int h, const orc_detect_params* p, orc_block_grid* g);

/* cv::circle(mask, Point(cvRound(x), cvRound(y)), r, 0, FILLED) for every point;
   mask must be pre-filled by the caller. */
void orc_mask_circles(uint8_t* mask, int w, int h, const float* xy, int n, int radius);

/* cornerMinEigenVal(blockSize 3, ksize 3) of the ROI [x0,x0+rw)x[y0,y0+rh) of the
   w x h image: Sobel reads the parent image across the ROI edge, the box filter
   reflects inside the ROI.  eig is rw*rh floats. */
void orc_corner_min_eigen_val(const uint8_t* img, int w, int h, int stride, int x0, int y0, int rw,
                              int rh, float* eig);

/* goodFeaturesToTrack on the ROI with mask ROI; returns the number of corners (ROI
   coordinates, integer-valued floats). */
int orc_good_features_to_track(const uint8_t* img, int w, int h, int stride, int x0, int y0, int rw,
                               int rh, const uint8_t* mask, int mask_stride, int max_corners,
                               double quality, double min_distance, float* out_xy);

/* cornerSubPix on the ROI (ROI coordinates in/out). */
void orc_corner_subpix(const uint8_t* img, int stride, int x0, int y0, int rw, int rh, float* xy,
                       int n, int win, int max_iters, double eps);

/* Tracking::featuresDetection (tracking.cc:576-688) on one frame.
   count_xy: points counted per block (frame->features() key points + pts2d_new_).
   mask_xy:  points masked with circles (frame_cur_->features() + pts2d_new_).
   n_existing: num_features for the early-exit test (features + pts2d_ref_).
   Outputs new corners in image coordinates, block-major; per-block counts.
   Returns the number of new corners, or -1 if the early exit triggered. */
int orc_features_detection(const uint8_t* img, int w, int h, int stride, const float* count_xy,
                           int n_count, const float* mask_xy, int n_mask, int ismask, int n_existing,
                           const orc_detect_params* p, float* out_xy, int* out_block_counts);

/* ------------------------------------------------------------------------- */
/* IMU preintegration (fp64)                                                  */
/* ------------------------------------------------------------------------- */

enum { ORC_PREINT_NORMAL = 0, ORC_PREINT_EARTH = 2 };

/* IMU record, types.h:50-58: {time, dt, dtheta[3], dvel[3], odovel}. */
typedef struct {
    double time, dt, dtheta[3], dvel[3], odovel;
} orc_imu;

/* IntegrationParameters (integration_state.h:68-89) subset used on the path. */
typedef struct {
    double acc_vrw, gyr_arw, gyr_bias_std, acc_bias_std, corr_time, gravity;
} orc_imu_params;

/* IntegrationState core (integration_state.h:35-51); q stored (x, y, z, w). */
typedef struct {
    double time;
    double p[3], q[4], v[3], bg[3], ba[3];
} orc_state;

/* Everything a PreintegrationBase holds after integrating a segment. */
typedef struct {
    int variant, m;          /* m = number of IMU records (imu_buffer_.size()) */
    double delta_time, start_time, end_time;
    orc_state current, delta;
    double gravity[3];
    double jacobian[225];    /* row-major 15x15 */
    double covariance[225];
    double noise[144];       /* 12x12 */
    double q0[4], iewn[3];   /* Earth variant only */
    double* pn;              /* (m-1) x {dt, p[3]}; Earth variant only */
} orc_preint;

/* Preintegration::createPreintegration + addNewImu for k = 1..m-1
   (ic_gvins.cc:946-953).  iewn is the Earth rate computed by the caller exactly
   as resetState does (orc_earth_iewn).  pn buffer is allocated. */
void orc_preint_integrate(orc_preint* s, int variant, const orc_imu_params* prm, const orc_imu* imu,
                          int m, const orc_state* state0, const double iewn[3]);
/* PreintegrationBase::reintegration (preintegration_base.cc:77-84). */
void orc_preint_reintegrate(orc_preint* s, const orc_imu_params* prm, const orc_imu* imu,
                            const orc_state* state, const double iewn[3]);
void orc_preint_free(orc_preint* s);

/* PreintegrationFactor::Evaluate: params = {pose0[7], mix0[9], pose1[7], mix1[9]};
   jac[i] may be NULL; jac == NULL means residual only.  Mutates s->corrected_* like
   the reference does (kept internal). */
void orc_preint_factor_eval(const orc_preint* s, const double* const* params, double* residual,
                            double** jac);

/* Earth::iewn(origin, local) (earth.h:233-237) via local2global/ecef2blh. */
void orc_earth_iewn(const double origin[3], const double local[3], double iewn[3]);

/* ------------------------------------------------------------------------- */
/* Reprojection factor                                                        */
/* ------------------------------------------------------------------------- */

/* Constants of one ReprojectionFactor (reprojection_factor.h:47-58). */
typedef struct {
    double pts0[3], pts1[3], vel0[3], vel1[3], td0, td1, std;
} orc_reproj_const;

/* params = {pose_ref[7], pose_obs[7], ext[7], invdepth[1], td[1]}; jac[i] may be
   NULL (2x7, 2x7, 2x7, 2x1, 2x1 row-major). */
void orc_reproj_eval(const orc_reproj_const* c, const double* const* params, double* residual,
                     double** jac);

/* CPU baseline of a solve's factor evaluation (the reference evaluates with
   Ceres num_threads = 4, ic_gvins.cc:1180): n reprojection factors over packed
   parameters (factor i: blocks at params + offs[5i+k]); residuals n x 2,
   jacobians (may be NULL) n x 46 = [J0 | J1 | J2 | J3 | J4]. */
void orc_reproj_eval_batch(int n, const orc_reproj_const* c, const double* params, const int* offs,
                           double* residuals, double* jacobians, int nthreads);
/* n preintegration factors (segments segs[i], blocks at params + offs[4i+k]);
   residuals n x 15, jacobians (may be NULL) n x 480. */
void orc_preint_factor_eval_batch(int n, const orc_preint* const* segs, const double* params, const int* offs,
                                  double* residuals, double* jacobians, int nthreads);

/* PoseParameterization::Plus (pose_parameterization.h:34-49). */
void orc_pose_plus(const double* x, const double* delta, double* x_plus_delta);

/* ------------------------------------------------------------------------- */
/* Preprocessing: CLAHE and the histogram check (clahe.c)                     */
/* ------------------------------------------------------------------------- */
/* cv::cvtColor(src, dst, COLOR_BGR2GRAY) for 8-bit BGR (OpenCV 4.x RGB2Gray<uchar>:
   (B*1868 + G*9617 + R*4899 + (1 << 13)) >> 14); the reference converts BGR8
   frames this way first (tracking.cc:111-113). */
void orc_bgr2gray(const uint8_t* bgr, int w, int h, int stride, uint8_t* gray, int gray_stride);
void orc_clahe_geometry(int w, int h, int tiles_x, int tiles_y, int* tw, int* th, int* ext_w, int* ext_h);
void orc_clahe_luts(const uint8_t* src, int w, int h, int stride, double clip_limit, int tiles_x,
                    int tiles_y, uint8_t* lut);
void orc_clahe(const uint8_t* src, int w, int h, int stride, double clip_limit, int tiles_x, int tiles_y,
               uint8_t* dst, int dst_stride);
double orc_hist_mean(const uint8_t* src, int w, int h, int stride);

/* ------------------------------------------------------------------------- */
/* INS mechanization (ins.c)                                                  */
/* ------------------------------------------------------------------------- */
/* IntegrationConfiguration (integration_state.h:91-99) as the mechanization
   reads it; iswithscale is false in the reference (ic_gvins.cc:116). */
typedef struct {
    int iswithearth;
    double gravity[3];  /* (0, 0, g) */
    double iewn[3];     /* Earth::iewn(origin, p), ic_gvins.cc:709-711 */
} orc_ins_config;
void orc_ins_mechanization(const orc_ins_config* cfg, const orc_imu* pre, const orc_imu* cur, orc_state* s);
void orc_ins_propagate(const orc_ins_config* cfg, const orc_imu* imu, int m, const orc_state* state0,
                       orc_state* states);
int orc_ins_window_index(const orc_imu* imu, int n, double t);
int orc_need_interpolation(const orc_imu* imu0, const orc_imu* imu1, double mid);
void orc_imu_interpolation(const orc_imu* imu01, orc_imu* imu00, orc_imu* imu11, double mid);
/* returns the window index (0: not found, nothing written) */
int orc_redo_ins_mechanization(const orc_ins_config* cfg, const orc_state* updated, const orc_imu* imu, int n,
                               orc_state* states);
/* returns the series length (<= n + 2), -1 when the window does not cover it */
int orc_imu_series_from_to(const orc_imu* imu, int n, double start, double end, orc_imu* series);

/* ------------------------------------------------------------------------- */
/* Remaining window factors (aux_factors.c)                                   */
/* ------------------------------------------------------------------------- */
/* kind 0 GNSS, 1 IMU_ERROR, 2 POSE_PRIOR, 3 MIX_PRIOR; dims = {residuals,
   parameter block size, constants per factor}.  Returns -1 for a bad kind. */
extern const int orc_small_factor_dims[4][3];
int orc_small_factor_eval(int kind, int n, const double* consts, const double* params, const int* offs,
                          double* residuals, double* jacobians);
/* J0 column-major r x r; block b: size[b] (7 = pose), index[b] (dx offset),
   xoff[b] (offset of its values in x0 / params and of its Jacobian, r * xoff[b]) */
void orc_marg_factor_eval(int r, int nb, const int* size, const int* index, const int* xoff, const double* x0,
                          const double* params, const double* J0, const double* e0, double* residuals,
                          double* jacobians);

/* ------------------------------------------------------------------------- */
/* Marginalisation (marg.c): MarginalizationInfo::constructEquation /         */
/* schurElimination / linearization and Eigen's SelfAdjointEigenSolver        */
/* ------------------------------------------------------------------------- */
/* A column-major (ld lda), lower triangle read -> eigenvalues w ascending,
   eigenvectors V (n x n column-major).  Returns 0, or 1 on NoConvergence. */
int orc_sym_eigen(int n, const double* A, int lda, double* w, double* V);
/* factor f: residuals then per block the row-major nres x size Jacobian at
   data + fac_off[f]; blocks blk[blk_off[f] .. blk_off[f+1]); loss[f] > 0: HuberLoss
   parameter (nullable).  H0 L x L column-major, b0 [L]. */
void orc_marg_construct(int n_fac, const int* nres, const int* blk_off, const int* blk, const long* fac_off,
                        const double* data, const double* loss, const int* size, const int* index, int L,
                        double* H0, double* b0);
/* Hp r x r column-major, bp [r], r = L - m.  Returns the eigen-solver info. */
int orc_marg_schur(int L, int m, const double* H0, const double* b0, double* Hp, double* bp);
/* J0 r x r column-major, e0 [r], eval [r] (nullable): Hp's eigenvalues */
int orc_marg_linearize(int r, const double* Hp, const double* bp, double* J0, double* e0, double* eval);

/* ------------------------------------------------------------------------- */
/* cv::findFundamentalMat(FM_RANSAC) (fmat.c, tracking.cc:547-548)            */
/* ------------------------------------------------------------------------- */
/* count >= 15 float2 point pairs -> mask (1 = inlier); returns 1 (model found),
   0 (none: mask zeroed), -1 (count < 15: OpenCV would run LMeDS, not modelled).
   F (nullable): the best model, row-major; iters_out (nullable): iterations run. */
int orc_find_fundamental_ransac(int count, const float* m1, const float* m2, double thresh, double confidence,
                                int max_iters, unsigned char* mask, double* F, int* iters_out);
int orc_run7point(const float* m1, const float* m2, double* F);       /* up to 3 models */
int orc_solve_cubic(const double* coeffs, double* roots);
void orc_fm_error(int n, const float* m1, const float* m2, const double* F, float* err);
int orc_ransac_update_num_iters(double p, double ep, int model_points, int max_iters);
unsigned orc_cvrng_next(uint64_t* state);

/* ------------------------------------------------------------------------- */
/* Camera operations (camera.c)                                               */
/* ------------------------------------------------------------------------- */
typedef struct {
    double fx, fy, cx, cy, skew;  /* intrinsic [fx skew cx; 0 fy cy; 0 0 1] (camera.cc:29-33) */
    double k1, k2, p1, p2, k3;    /* distortion (camera.cc:35-39) */
    int width, height;
} orc_camera;
void orc_undistort_points(const orc_camera* c, int n, const float* in, float* out);
void orc_distort_points(const orc_camera* c, int n, const float* in, float* out);
void orc_predict_rotated(const orc_camera* c, const double* r_cur_pre, int n, const float* in, float* out);
void orc_project_points(const orc_camera* c, const double* R, const double* t, int n, const double* pw,
                        float* out);
void orc_point_velocity(const orc_camera* c, int n, const float* pre, const float* cur, double dt, double* vel);
void orc_r1t_r0(const double* R0, const double* R1, double* M);
void orc_keypoint_parallax(const orc_camera* c, const double* R0, const double* R1, int n, const float* ref,
                           const float* cur, double* out);

#ifdef __cplusplus
}
#endif

#endif /* GVX_ORACLE_H */
