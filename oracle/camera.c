/*
 * camera.c -- CPU restatement of the per-point camera operations around the
 * KLT calls (TEST INFRASTRUCTURE ONLY; see gvx_oracle.h).  Paths relative to
 * /root/reference/ic_gvins/ic_gvins/.
 *
 *   orc_undistort_points   Camera::undistortPoints (tracking/camera.cc:72-74) =
 *                          cv::undistortPoints(pts, pts, K, D, Mat(), K), OpenCV 4.x
 *                          cvUndistortPointsInternal with the default criteria
 *                          (COUNT, 5 iterations): x = (u - cx)/fx (as u*ifx,
 *                          ifx = 1./fx; the skew is not used), 5 fixed-point steps
 *                          x = (x0 - delta(x)) * icdist(x), the icdist < 0 escape,
 *                          then (x, y) -> P (fx*x + skew*y + cx, fy*y + cy).
 *   orc_distort_points     Camera::distortPoints (camera.cc:76-89): pixel2cam
 *                          (:122-126), radial-tangential model, cam2pixel (:129-131).
 *   orc_predict_rotated    Tracking::trackReferenceFrame's rotation-compensated
 *                          initial flow (tracking/tracking.cc:465-478): undistort,
 *                          pixel2cam, r_cur_pre * pc, distortCameraPoint
 *                          (camera.cc:105-118, float-rounded normalised point).
 *   orc_project_points     Tracking::trackMappoint's prediction (tracking.cc:366-377):
 *                          world2pixel (camera.cc:137-143) then distortPoints.
 *   orc_point_velocity     (pixel2cam(cur) - pixel2cam(pre)) / dt
 *                          (tracking.cc:433, :530).
 *   orc_keypoint_parallax  Tracking::keyPointParallax (tracking.cc:861-871) with
 *                          M = R1^T R0 (Eigen evaluates the nested product into a
 *                          temporary first) and focalLength = (fx + fy) * 0.5
 *                          (camera.h:82-84).
 *
 * Eigen 3x3 products are restated as ((a0 + a1) + a2) per coefficient; every
 * expression is evaluated left to right without FMA contraction.
 * Parity unpinned: OpenCV/Eigen are absent here; pinned by the round-trip and
 * known-answer tests in tests/test_oracle_camera.py.
 */
#include <math.h>

#include "gvx_oracle.h"

static void pixel2cam(const orc_camera* c, float px, float py, double* x, double* y) {
    const double yy = ((double)py - c->cy) / c->fy;
    *y = yy;
    *x = ((double)px - c->cx - c->skew * yy) / c->fx;
}

static void cam2pixel(const orc_camera* c, double x, double y, double z, float* px, float* py) {
    *px = (float)((c->fx * x + c->skew * y) / z + c->cx);
    *py = (float)(c->fy * y / z + c->cy);
}

static void distort_norm(const orc_camera* c, double x, double y, double* ox, double* oy) {
    const double r2 = x * x + y * y;
    const double rr = (1 + c->k1 * r2 + c->k2 * r2 * r2 + c->k3 * r2 * r2 * r2);
    *ox = x * rr + 2 * c->p1 * x * y + c->p2 * (r2 + 2 * x * x);
    *oy = y * rr + c->p1 * (r2 + 2 * y * y) + 2 * c->p2 * x * y;
}

static void mat3_vec(const double* M, double x, double y, double z, double* o) {
    for (int i = 0; i < 3; ++i) o[i] = M[3 * i] * x + M[3 * i + 1] * y + M[3 * i + 2] * z;
}

void orc_undistort_points(const orc_camera* c, int n, const float* in, float* out) {
    const double ifx = 1. / c->fx, ify = 1. / c->fy;
    for (int i = 0; i < n; ++i) {
        double x = in[2 * i], y = in[2 * i + 1];
        const double u = x, v = y;
        x = (x - c->cx) * ifx;
        y = (y - c->cy) * ify;
        const double x0 = x, y0 = y;
        for (int j = 0; j < 5; ++j) {
            const double r2 = x * x + y * y;
            const double icdist = 1 / (1 + ((c->k3 * r2 + c->k2) * r2 + c->k1) * r2);
            if (icdist < 0) {
                x = (u - c->cx) * ifx;
                y = (v - c->cy) * ify;
                break;
            }
            const double dx = 2 * c->p1 * x * y + c->p2 * (r2 + 2 * x * x);
            const double dy = c->p1 * (r2 + 2 * y * y) + 2 * c->p2 * x * y;
            x = (x0 - dx) * icdist;
            y = (y0 - dy) * icdist;
        }
        const double xx = c->fx * x + c->skew * y + c->cx;
        const double yy = c->fy * y + c->cy;
        out[2 * i] = (float)xx;
        out[2 * i + 1] = (float)yy;
    }
}

void orc_distort_points(const orc_camera* c, int n, const float* in, float* out) {
    for (int i = 0; i < n; ++i) {
        double x, y, dx, dy;
        pixel2cam(c, in[2 * i], in[2 * i + 1], &x, &y);
        distort_norm(c, x, y, &dx, &dy);
        cam2pixel(c, dx, dy, 1.0, &out[2 * i], &out[2 * i + 1]);
    }
}

void orc_predict_rotated(const orc_camera* c, const double* r_cur_pre, int n, const float* in, float* out) {
    for (int i = 0; i < n; ++i) {
        float u[2];
        orc_undistort_points(c, 1, in + 2 * i, u);
        double x, y, pc[3], dx, dy;
        pixel2cam(c, u[0], u[1], &x, &y);
        mat3_vec(r_cur_pre, x, y, 1.0, pc);
        distort_norm(c, pc[0] / pc[2], pc[1] / pc[2], &dx, &dy);
        cam2pixel(c, (double)(float)dx, (double)(float)dy, 1.0, &out[2 * i], &out[2 * i + 1]);
    }
}

void orc_project_points(const orc_camera* c, const double* R, const double* t, int n, const double* pw,
                        float* out) {
    for (int i = 0; i < n; ++i) {
        const double d[3] = {pw[3 * i] - t[0], pw[3 * i + 1] - t[1], pw[3 * i + 2] - t[2]};
        double pc[3];
        for (int k = 0; k < 3; ++k) pc[k] = R[k] * d[0] + R[3 + k] * d[1] + R[6 + k] * d[2];  /* R^T d */
        float p[2];
        cam2pixel(c, pc[0], pc[1], pc[2], &p[0], &p[1]);
        orc_distort_points(c, 1, p, out + 2 * i);
    }
}

void orc_point_velocity(const orc_camera* c, int n, const float* pre, const float* cur, double dt, double* vel) {
    for (int i = 0; i < n; ++i) {
        double x0, y0, x1, y1;
        pixel2cam(c, pre[2 * i], pre[2 * i + 1], &x0, &y0);
        pixel2cam(c, cur[2 * i], cur[2 * i + 1], &x1, &y1);
        vel[2 * i] = (x1 - x0) / dt;
        vel[2 * i + 1] = (y1 - y0) / dt;
    }
}

void orc_r1t_r0(const double* R0, const double* R1, double* M) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) M[3 * i + j] = R1[i] * R0[j] + R1[3 + i] * R0[3 + j] + R1[6 + i] * R0[6 + j];
}

void orc_keypoint_parallax(const orc_camera* c, const double* R0, const double* R1, int n, const float* ref,
                           const float* cur, double* out) {
    double M[9];
    orc_r1t_r0(R0, R1, M);
    const double f = (c->fx + c->fy) * 0.5;
    for (int i = 0; i < n; ++i) {
        double x0, y0, x1, y1, p[3];
        pixel2cam(c, ref[2 * i], ref[2 * i + 1], &x0, &y0);
        pixel2cam(c, cur[2 * i], cur[2 * i + 1], &x1, &y1);
        mat3_vec(M, x0, y0, 1.0, p);
        const double dx = p[0] - x1, dy = p[1] - y1;
        out[i] = sqrt(dx * dx + dy * dy) * f;
    }
}
