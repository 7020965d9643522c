// camera.hip -- per-point camera operations around the KLT calls, for gfx950
// (paths relative to /root/reference/ic_gvins/ic_gvins/):
//   UNDISTORT  Camera::undistortPoints (tracking/camera.cc:72-74) =
//              cv::undistortPoints(pts, pts, K, D, Mat(), K), OpenCV 4.x, 5 steps
//   DISTORT    Camera::distortPoints (camera.cc:76-89)
//   PREDICT    Tracking::trackReferenceFrame's rotation-compensated initial flow
//              (tracking/tracking.cc:465-478)
//   PROJECT    Tracking::trackMappoint's prediction (tracking.cc:366-377)
//   VELOCITY   (pixel2cam(cur) - pixel2cam(pre)) / dt (tracking.cc:433, :530)
//   PARALLAX   Tracking::keyPointParallax (tracking.cc:861-871)
// One thread per point, fp64 in the CPU restatement's order (oracle/camera.c;
// built with -ffp-contract=off, IEEE division and square root), so the float
// pixel outputs are bit-identical to it.  The work is a few hundred flops per
// point on at most a few hundred points per frame: these kernels exist so a
// frame's tracking epilogue stays on the device, not for throughput.
#include <hip/hip_runtime.h>

#include "gvx_internal.h"

namespace gvx {

namespace {

__device__ __forceinline__ void pixel2cam(const gvx_camera& c, float px, float py, double& x, double& y) {
    const double yy = ((double)py - c.cy) / c.fy;
    y = yy;
    x = ((double)px - c.cx - c.skew * yy) / c.fx;
}

__device__ __forceinline__ float2 cam2pixel(const gvx_camera& c, double x, double y, double z) {
    return make_float2((float)((c.fx * x + c.skew * y) / z + c.cx), (float)(c.fy * y / z + c.cy));
}

__device__ __forceinline__ void distort_norm(const gvx_camera& c, double x, double y, double& ox, double& oy) {
    const double r2 = x * x + y * y;
    const double rr = (1 + c.k1 * r2 + c.k2 * r2 * r2 + c.k3 * r2 * r2 * r2);
    ox = x * rr + 2 * c.p1 * x * y + c.p2 * (r2 + 2 * x * x);
    oy = y * rr + c.p1 * (r2 + 2 * y * y) + 2 * c.p2 * x * y;
}

__device__ __forceinline__ float2 undistort(const gvx_camera& c, float2 p) {
    const double ifx = 1. / c.fx, ify = 1. / c.fy;
    const double u = p.x, v = p.y;
    double x = (u - c.cx) * ifx, y = (v - c.cy) * ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; ++j) {
        const double r2 = x * x + y * y;
        const double icdist = 1 / (1 + ((c.k3 * r2 + c.k2) * r2 + c.k1) * r2);
        if (icdist < 0) {
            x = (u - c.cx) * ifx;
            y = (v - c.cy) * ify;
            break;
        }
        const double dx = 2 * c.p1 * x * y + c.p2 * (r2 + 2 * x * x);
        const double dy = c.p1 * (r2 + 2 * y * y) + 2 * c.p2 * x * y;
        x = (x0 - dx) * icdist;
        y = (y0 - dy) * icdist;
    }
    return make_float2((float)(c.fx * x + c.skew * y + c.cx), (float)(c.fy * y + c.cy));
}

__device__ __forceinline__ float2 distort(const gvx_camera& c, float2 p) {
    double x, y, dx, dy;
    pixel2cam(c, p.x, p.y, x, y);
    distort_norm(c, x, y, dx, dy);
    return cam2pixel(c, dx, dy, 1.0);
}

template <int OP>
__global__ void __launch_bounds__(256) camera_kernel(CamArgs a, const void* __restrict__ in0,
                                                     const void* __restrict__ in1, void* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    const gvx_camera& c = a.cam;
    if constexpr (OP == GVX_CAM_UNDISTORT || OP == GVX_CAM_DISTORT || OP == GVX_CAM_PREDICT) {
        const float2 p = reinterpret_cast<const float2*>(in0)[i];
        float2 r;
        if constexpr (OP == GVX_CAM_UNDISTORT) {
            r = undistort(c, p);
        } else if constexpr (OP == GVX_CAM_DISTORT) {
            r = distort(c, p);
        } else {
            const float2 u = undistort(c, p);
            double x, y, dx, dy;
            pixel2cam(c, u.x, u.y, x, y);
            double pc[3];
            for (int k = 0; k < 3; ++k) pc[k] = a.M[3 * k] * x + a.M[3 * k + 1] * y + a.M[3 * k + 2] * 1.0;
            distort_norm(c, pc[0] / pc[2], pc[1] / pc[2], dx, dy);
            r = cam2pixel(c, (double)(float)dx, (double)(float)dy, 1.0);
        }
        reinterpret_cast<float2*>(out)[i] = r;
    } else if constexpr (OP == GVX_CAM_PROJECT) {
        const double* pw = reinterpret_cast<const double*>(in0) + 3 * i;
        const double d[3] = {pw[0] - a.t[0], pw[1] - a.t[1], pw[2] - a.t[2]};
        double pc[3];
        for (int k = 0; k < 3; ++k) pc[k] = a.M[k] * d[0] + a.M[3 + k] * d[1] + a.M[6 + k] * d[2];  // R^T d
        reinterpret_cast<float2*>(out)[i] = distort(c, cam2pixel(c, pc[0], pc[1], pc[2]));
    } else {
        const float2 p0 = reinterpret_cast<const float2*>(in0)[i];
        const float2 p1 = reinterpret_cast<const float2*>(in1)[i];
        double x0, y0, x1, y1;
        pixel2cam(c, p0.x, p0.y, x0, y0);
        pixel2cam(c, p1.x, p1.y, x1, y1);
        if constexpr (OP == GVX_CAM_VELOCITY) {
            double* v = reinterpret_cast<double*>(out) + 2 * i;
            v[0] = (x1 - x0) / a.dt;
            v[1] = (y1 - y0) / a.dt;
        } else {
            double p[3];
            for (int k = 0; k < 3; ++k) p[k] = a.M[3 * k] * x0 + a.M[3 * k + 1] * y0 + a.M[3 * k + 2] * 1.0;
            const double dx = p[0] - x1, dy = p[1] - y1;
            reinterpret_cast<double*>(out)[i] = __dsqrt_rn(dx * dx + dy * dy) * ((c.fx + c.fy) * 0.5);
        }
    }
}

template <int OP>
void launch_op(gvx_ctx* c, const CamArgs& a, const void* in0, const void* in1, void* out) {
    hipLaunchKernelGGL(camera_kernel<OP>, dim3((a.n + 255) / 256), dim3(256), 0, c->stream, a, in0, in1, out);
}

}  // namespace

hipError_t launch_camera(gvx_ctx* c, int op, const CamArgs& a, const void* in0, const void* in1, void* out) {
    if (a.n <= 0) return hipSuccess;
    switch (op) {
        case GVX_CAM_UNDISTORT: launch_op<GVX_CAM_UNDISTORT>(c, a, in0, in1, out); break;
        case GVX_CAM_DISTORT: launch_op<GVX_CAM_DISTORT>(c, a, in0, in1, out); break;
        case GVX_CAM_PREDICT: launch_op<GVX_CAM_PREDICT>(c, a, in0, in1, out); break;
        case GVX_CAM_PROJECT: launch_op<GVX_CAM_PROJECT>(c, a, in0, in1, out); break;
        case GVX_CAM_VELOCITY: launch_op<GVX_CAM_VELOCITY>(c, a, in0, in1, out); break;
        case GVX_CAM_PARALLAX: launch_op<GVX_CAM_PARALLAX>(c, a, in0, in1, out); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace gvx
