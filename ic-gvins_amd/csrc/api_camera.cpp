// api_camera.cpp -- C ABI of the per-point camera operations (include/gvx.h):
// Camera (/root/reference/ic_gvins/ic_gvins/tracking/camera.cc) and the point
// epilogues of Tracking::trackMappoint / trackReferenceFrame (tracking.cc:351-574).
#include <cmath>
#include <cstring>

#include "gvx_internal.h"

using namespace gvx;

static gvx_status check_cam(gvx_ctx* c, const gvx_camera* cam, int32_t n) {
    if (!cam) return set_err(c, GVX_ERR_INVALID, "null camera");
    if (n < 0) return set_err(c, GVX_ERR_INVALID, "negative point count");
    if (!(cam->fx != 0.0 && cam->fy != 0.0 && std::isfinite(cam->fx) && std::isfinite(cam->fy)))
        return set_err(c, GVX_ERR_INVALID, "camera focal lengths must be finite and non-zero");
    return GVX_OK;
}

static CamArgs cam_args(const gvx_camera* cam, const double* M, const double* t, double dt, int n) {
    CamArgs a{};
    a.cam = *cam;
    if (M) std::memcpy(a.M, M, sizeof a.M);
    if (t) std::memcpy(a.t, t, sizeof a.t);
    a.dt = dt;
    a.n = n;
    return a;
}

// pose1.R.transpose() * pose0.R (keyPointParallax's nested product, evaluated
// first into a temporary by Eigen), ((a0 + a1) + a2) per coefficient.
static void r1t_r0(const double* R0, const double* R1, double* M) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) M[3 * i + j] = R1[i] * R0[j] + R1[3 + i] * R0[3 + j] + R1[6 + i] * R0[6 + j];
}

static gvx_status dev_op(gvx_ctx* c, int op, const CamArgs& a, const void* in0, const void* in1, void* out) {
    if (a.n == 0) return GVX_OK;
    if (!in0 || !out || ((op == GVX_CAM_VELOCITY || op == GVX_CAM_PARALLAX) && !in1))
        return set_err(c, GVX_ERR_INVALID, "null point buffer");
    hipSetDevice(c->device);
    hipEvent_t ev{};
    prof_begin(c, "camera", &ev);
    hipError_t e = launch_camera(c, op, a, in0, in1, out);
    prof_end(c, "camera", ev);
    return hip_err(c, e, "camera kernel");
}

// Host form: stage in0 (b0 bytes) and in1 (b1 bytes), run, copy bo bytes back.
static gvx_status host_op(gvx_ctx* c, int op, const CamArgs& a, const void* in0, size_t b0, const void* in1,
                          size_t b1, void* out, size_t bo) {
    if (a.n == 0) return GVX_OK;
    if (!in0 || !out || (b1 && !in1)) return set_err(c, GVX_ERR_INVALID, "null point buffer");
    hipSetDevice(c->device);
    const size_t tot = b0 + b1 + bo;
    uint8_t* h = (uint8_t*)pinned(c, "cam_io", tot);
    uint8_t* d = (uint8_t*)scratch(c, "cam_io", tot);
    if (!h || !d) return set_err(c, GVX_ERR_OOM, "camera staging");
    hipStreamSynchronize(c->stream);  // staging buffer reuse
    std::memcpy(h, in0, b0);
    if (b1) std::memcpy(h + b0, in1, b1);
    hipError_t e = hipMemcpyAsync(d, h, b0 + b1, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "hipMemcpyAsync(points)");
    gvx_status s = dev_op(c, op, a, d, b1 ? d + b0 : nullptr, d + b0 + b1);
    if (s) return s;
    e = hipMemcpyAsync(h + b0 + b1, d + b0 + b1, bo, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "camera copy-out");
    std::memcpy(out, h + b0 + b1, bo);
    return GVX_OK;
}

#define GVX_CAM_CHECK(c, cam, n)               \
    if (!(c)) return GVX_ERR_INVALID;          \
    {                                          \
        gvx_status s_ = check_cam(c, cam, n);  \
        if (s_) return s_;                     \
    }

gvx_status gvx_undistort_points(gvx_ctx* c, const gvx_camera* cam, int32_t n, const float* xy, float* out) {
    GVX_CAM_CHECK(c, cam, n);
    return host_op(c, GVX_CAM_UNDISTORT, cam_args(cam, nullptr, nullptr, 0, n), xy, 8 * (size_t)n, nullptr, 0, out,
                   8 * (size_t)n);
}
gvx_status gvx_undistort_points_dev(gvx_ctx* c, const gvx_camera* cam, int32_t n, const float* d_xy, float* d_out) {
    GVX_CAM_CHECK(c, cam, n);
    return dev_op(c, GVX_CAM_UNDISTORT, cam_args(cam, nullptr, nullptr, 0, n), d_xy, nullptr, d_out);
}

gvx_status gvx_distort_points(gvx_ctx* c, const gvx_camera* cam, int32_t n, const float* xy, float* out) {
    GVX_CAM_CHECK(c, cam, n);
    return host_op(c, GVX_CAM_DISTORT, cam_args(cam, nullptr, nullptr, 0, n), xy, 8 * (size_t)n, nullptr, 0, out,
                   8 * (size_t)n);
}
gvx_status gvx_distort_points_dev(gvx_ctx* c, const gvx_camera* cam, int32_t n, const float* d_xy, float* d_out) {
    GVX_CAM_CHECK(c, cam, n);
    return dev_op(c, GVX_CAM_DISTORT, cam_args(cam, nullptr, nullptr, 0, n), d_xy, nullptr, d_out);
}

gvx_status gvx_predict_rotated(gvx_ctx* c, const gvx_camera* cam, const double* r_cur_pre, int32_t n,
                               const float* xy, float* out) {
    GVX_CAM_CHECK(c, cam, n);
    if (!r_cur_pre) return set_err(c, GVX_ERR_INVALID, "null rotation");
    return host_op(c, GVX_CAM_PREDICT, cam_args(cam, r_cur_pre, nullptr, 0, n), xy, 8 * (size_t)n, nullptr, 0, out,
                   8 * (size_t)n);
}
gvx_status gvx_predict_rotated_dev(gvx_ctx* c, const gvx_camera* cam, const double* r_cur_pre, int32_t n,
                                   const float* d_xy, float* d_out) {
    GVX_CAM_CHECK(c, cam, n);
    if (!r_cur_pre) return set_err(c, GVX_ERR_INVALID, "null rotation");
    return dev_op(c, GVX_CAM_PREDICT, cam_args(cam, r_cur_pre, nullptr, 0, n), d_xy, nullptr, d_out);
}

gvx_status gvx_project_points(gvx_ctx* c, const gvx_camera* cam, const double* R, const double* t, int32_t n,
                              const double* pw, float* out) {
    GVX_CAM_CHECK(c, cam, n);
    if (!R || !t) return set_err(c, GVX_ERR_INVALID, "null pose");
    return host_op(c, GVX_CAM_PROJECT, cam_args(cam, R, t, 0, n), pw, 24 * (size_t)n, nullptr, 0, out,
                   8 * (size_t)n);
}
gvx_status gvx_project_points_dev(gvx_ctx* c, const gvx_camera* cam, const double* R, const double* t, int32_t n,
                                  const double* d_pw, float* d_out) {
    GVX_CAM_CHECK(c, cam, n);
    if (!R || !t) return set_err(c, GVX_ERR_INVALID, "null pose");
    return dev_op(c, GVX_CAM_PROJECT, cam_args(cam, R, t, 0, n), d_pw, nullptr, d_out);
}

gvx_status gvx_point_velocity(gvx_ctx* c, const gvx_camera* cam, int32_t n, const float* pre, const float* cur,
                              double dt, double* vel) {
    GVX_CAM_CHECK(c, cam, n);
    return host_op(c, GVX_CAM_VELOCITY, cam_args(cam, nullptr, nullptr, dt, n), pre, 8 * (size_t)n, cur,
                   8 * (size_t)n, vel, 16 * (size_t)n);
}
gvx_status gvx_point_velocity_dev(gvx_ctx* c, const gvx_camera* cam, int32_t n, const float* d_pre,
                                  const float* d_cur, double dt, double* d_vel) {
    GVX_CAM_CHECK(c, cam, n);
    return dev_op(c, GVX_CAM_VELOCITY, cam_args(cam, nullptr, nullptr, dt, n), d_pre, d_cur, d_vel);
}

gvx_status gvx_keypoint_parallax(gvx_ctx* c, const gvx_camera* cam, const double* R0, const double* R1, int32_t n,
                                 const float* ref, const float* cur, double* out) {
    GVX_CAM_CHECK(c, cam, n);
    if (!R0 || !R1) return set_err(c, GVX_ERR_INVALID, "null pose");
    double M[9];
    r1t_r0(R0, R1, M);
    return host_op(c, GVX_CAM_PARALLAX, cam_args(cam, M, nullptr, 0, n), ref, 8 * (size_t)n, cur, 8 * (size_t)n,
                   out, 8 * (size_t)n);
}
gvx_status gvx_keypoint_parallax_dev(gvx_ctx* c, const gvx_camera* cam, const double* R0, const double* R1,
                                     int32_t n, const float* d_ref, const float* d_cur, double* d_out) {
    GVX_CAM_CHECK(c, cam, n);
    if (!R0 || !R1) return set_err(c, GVX_ERR_INVALID, "null pose");
    double M[9];
    r1t_r0(R0, R1, M);
    return dev_op(c, GVX_CAM_PARALLAX, cam_args(cam, M, nullptr, 0, n), d_ref, d_cur, d_out);
}
