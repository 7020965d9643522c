// aux_factors.hip -- the remaining Ceres cost functions of the sliding window
// for gfx950 (fp64), beside the reprojection / preintegration kernels of
// factors.hip:
//   GnssFactor::Evaluate            factors/gnss_factor.h:52-95
//   ImuErrorFactor::Evaluate        preintegration/imu_error_factor.h:45-66
//   ImuPosePriorFactor::Evaluate    preintegration/imu_pose_prior_factor.h:42-68
//   ImuMixPriorFactor::Evaluate     preintegration/imu_mix_prior_factor.h:40-56
//   MarginalizationFactor::Evaluate factors/marginalization_factor.h:54-110
// (paths under /root/reference/ic_gvins/ic_gvins/).  Expressions follow the CPU
// restatement (oracle/aux_factors.c) in order, no FMA contraction.
//
// small_kernel<KIND>: one thread per factor; a few dozen flops and at most 81
//   Jacobian doubles each -- these factors number one per GNSS epoch / window,
//   so the kernel is there to keep a whole-iteration offload on the device.
// marg_kernel: one workgroup per marginalisation factor: dx of the remained
//   blocks into LDS, then e0 + J0 dx with thread i walking row i of the
//   column-major J0 (coalesced over i), then the Jacobian blocks copied out of
//   J0's columns -- HBM-bound on the r^2 doubles of J0.
#include <hip/hip_runtime.h>

#include "dmath.h"
#include "gvx_internal.h"

namespace gvx {

namespace {

constexpr double PI_D = 3.14159265358979323846;
constexpr double IMU_GRY_BIAS_STD = 7200 / 3600.0 * PI_D / 180.0;  // imu_error_factor.h:89
constexpr double IMU_ACC_BIAS_STD = 2.0e4 * 1.0e-5;                 // imu_error_factor.h:90

template <int KIND>
struct Dims;
template <>
struct Dims<GVX_FACTOR_GNSS> {
    static constexpr int R = 3, P = 7, NC = 9;
};
template <>
struct Dims<GVX_FACTOR_IMU_ERROR> {
    static constexpr int R = 6, P = 9, NC = 0;
};
template <>
struct Dims<GVX_FACTOR_POSE_PRIOR> {
    static constexpr int R = 6, P = 7, NC = 13;
};
template <>
struct Dims<GVX_FACTOR_MIX_PRIOR> {
    static constexpr int R = 9, P = 9, NC = 18;
};

template <int KIND>
__global__ void __launch_bounds__(64) small_kernel(int n, const double* __restrict__ consts,
                                                   const double* __restrict__ params, const int32_t* __restrict__ offs,
                                                   double* __restrict__ residuals, double* __restrict__ jacobians) {
    constexpr int R = Dims<KIND>::R, P = Dims<KIND>::P, NC = Dims<KIND>::NC;
    // outputs staged through LDS so the block's residual and Jacobian ranges
    // are stored contiguously (a thread's own 21-81 doubles would be strided)
    __shared__ double sres[64 * R], sjac[64 * R * P];
    const int lane = threadIdx.x, i0 = blockIdx.x * 64, i = i0 + lane;
    const int cnt = min(64, n - i0);
    double res[R], jac[R * P];
#pragma unroll
    for (int k = 0; k < R; ++k) res[k] = 0.0;
#pragma unroll
    for (int k = 0; k < R * P; ++k) jac[k] = 0.0;
    const double* c = consts + (int64_t)min(i, n - 1) * NC;
    const double* p = params + offs[min(i, n - 1)];
    if (i >= n) {
        // no factor: the stores below skip this lane's slots
    } else if constexpr (KIND == GVX_FACTOR_GNSS) {
        const double *blh = c, *stdv = c + 3, *lever = c + 6;
        const dq q = dq_make(p[6], p[3], p[4], p[5]);
        double Rm[9], Rl[3], s[3];
        dq_rot(q, Rm);
        mv3(Rm, lever, Rl);
        for (int k = 0; k < 3; ++k) s[k] = 1.0 / stdv[k];
        for (int k = 0; k < 3; ++k) res[k] = s[k] * (p[k] + Rl[k] - blh[k]);
        double nR[9], S[9], B[9];
        for (int k = 0; k < 9; ++k) nR[k] = -Rm[k];
        skew(lever, S);
        mm3(nR, S, B);
        for (int r = 0; r < 3; ++r) {
            jac[r * 7 + r] = s[r] * 1.0;
            for (int j = 0; j < 3; ++j) jac[r * 7 + 3 + j] = s[r] * B[r * 3 + j];
        }
    } else if constexpr (KIND == GVX_FACTOR_IMU_ERROR) {
        for (int k = 0; k < 3; ++k) {
            res[k] = p[k + 3] / IMU_GRY_BIAS_STD;
            res[k + 3] = p[k + 6] / IMU_ACC_BIAS_STD;
            jac[k * 9 + k + 3] = 1.0 / IMU_GRY_BIAS_STD;
            jac[(k + 3) * 9 + k + 6] = 1.0 / IMU_ACC_BIAS_STD;
        }
    } else if constexpr (KIND == GVX_FACTOR_POSE_PRIOR) {
        const double *prior = c, *stdv = c + 7;
        double r6[6], s[6];
        for (int k = 0; k < 3; ++k) r6[k] = p[k] - prior[k];
        const dq qp = dq_make(prior[6], prior[3], prior[4], prior[5]);
        const dq q = dq_make(p[6], p[3], p[4], p[5]);
        const dq d = dq_mul(dq_inv(q), qp);
        r6[3] = 2 * d.x;
        r6[4] = 2 * d.y;
        r6[5] = 2 * d.z;
        for (int k = 0; k < 6; ++k) s[k] = 1.0 / stdv[k];
        for (int k = 0; k < 6; ++k) res[k] = s[k] * r6[k];
        double M[9];
        qright_br(d, M);
        for (int k = 0; k < 3; ++k) jac[k * 7 + k] = s[k] * 1.0;
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) jac[(3 + a) * 7 + 3 + b] = s[3 + a] * -M[a * 3 + b];
    } else {
        const double *prior = c, *stdv = c + 9;
        for (int k = 0; k < 9; ++k) {
            res[k] = (p[k] - prior[k]) / stdv[k];
            jac[k * 9 + k] = 1.0 / stdv[k];
        }
    }
#pragma unroll
    for (int k = 0; k < R; ++k) sres[lane * R + k] = res[k];
    if (jacobians) {
#pragma unroll
        for (int k = 0; k < R * P; ++k) sjac[lane * R * P + k] = jac[k];
    }
    __syncthreads();
    double* ro = residuals + (int64_t)i0 * R;
    for (int k = lane; k < cnt * R; k += 64) __builtin_nontemporal_store(sres[k], ro + k);
    if (jacobians) {
        double* jo = jacobians + (int64_t)i0 * R * P;
        for (int k = lane; k < cnt * R * P; k += 64) __builtin_nontemporal_store(sjac[k], jo + k);
    }
}

constexpr int MARG_THREADS = 256;

__global__ void __launch_bounds__(MARG_THREADS) marg_kernel(int r, int nb, const int32_t* __restrict__ blk,
                                                            const double* __restrict__ x0,
                                                            const double* __restrict__ x,
                                                            const double* __restrict__ J0,
                                                            const double* __restrict__ e0,
                                                            double* __restrict__ residuals,
                                                            double* __restrict__ jacobians) {
    extern __shared__ double sdx[];  // r doubles
    const int32_t *size = blk, *index = blk + nb, *xoff = blk + 2 * nb;
    const int t = threadIdx.x;
    for (int b = t; b < nb; b += MARG_THREADS) {
        const double* xv = x + xoff[b];
        const double* z = x0 + xoff[b];
        const int id = index[b];
        if (size[b] == 7) {  // POSE_GLOBAL_SIZE
            const dq d = dq_mul(dq_inv(dq_make(z[6], z[3], z[4], z[5])), dq_make(xv[6], xv[3], xv[4], xv[5]));
            for (int k = 0; k < 3; ++k) sdx[id + k] = xv[k] - z[k];
            const double s = d.w < 0 ? -2.0 : 2.0;
            sdx[id + 3] = s * d.x;
            sdx[id + 4] = s * d.y;
            sdx[id + 5] = s * d.z;
        } else {
            for (int k = 0; k < size[b]; ++k) sdx[id + k] = xv[k] - z[k];
        }
    }
    __syncthreads();
    for (int i = t; i < r; i += MARG_THREADS) {
        double acc = 0.0;
        for (int j = 0; j < r; ++j) acc += J0[(int64_t)j * r + i] * sdx[j];
        residuals[i] = e0[i] + acc;
    }
    if (!jacobians) return;
    for (int b = 0; b < nb; ++b) {
        const int sz = size[b], local = sz == 7 ? 6 : sz, id = index[b];
        double* J = jacobians + (int64_t)r * xoff[b];
        for (int q = t; q < r * sz; q += MARG_THREADS) {
            const int i = q / sz, cc = q - i * sz;
            J[q] = cc < local ? J0[(int64_t)(id + cc) * r + i] : 0.0;
        }
    }
}

}  // namespace

int small_factor_dims(int kind, int* P, int* NC) {
    switch (kind) {
        case GVX_FACTOR_GNSS: *P = 7, *NC = 9; return 3;
        case GVX_FACTOR_IMU_ERROR: *P = 9, *NC = 0; return 6;
        case GVX_FACTOR_POSE_PRIOR: *P = 7, *NC = 13; return 6;
        case GVX_FACTOR_MIX_PRIOR: *P = 9, *NC = 18; return 9;
        default: return 0;
    }
}

hipError_t launch_small_factor(gvx_ctx* c, int kind, int n, const double* consts, const double* params,
                               const int32_t* offs, double* residuals, double* jacobians) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((n + 63) / 64), block(64);
    switch (kind) {
        case GVX_FACTOR_GNSS:
            return launch_timed(c, "aux_factor", small_kernel<GVX_FACTOR_GNSS>, grid, block, 0, n, consts, params, offs,
                                residuals, jacobians);
        case GVX_FACTOR_IMU_ERROR:
            return launch_timed(c, "aux_factor", small_kernel<GVX_FACTOR_IMU_ERROR>, grid, block, 0, n, consts, params, offs,
                                residuals, jacobians);
        case GVX_FACTOR_POSE_PRIOR:
            return launch_timed(c, "aux_factor", small_kernel<GVX_FACTOR_POSE_PRIOR>, grid, block, 0, n, consts, params, offs,
                                residuals, jacobians);
        default:
            return launch_timed(c, "aux_factor", small_kernel<GVX_FACTOR_MIX_PRIOR>, grid, block, 0, n, consts, params, offs,
                                residuals, jacobians);
    }
}

hipError_t launch_marg_factor(gvx_ctx* c, int r, int nb, const int32_t* blk, const double* x0, const double* x,
                              const double* J0, const double* e0, double* residuals, double* jacobians) {
    if (r <= 0) return hipSuccess;
    hipLaunchKernelGGL(marg_kernel, dim3(1), dim3(MARG_THREADS), sizeof(double) * r, c->stream, r, nb, blk, x0, x,
                       J0, e0, residuals, jacobians);
    return hipGetLastError();
}

}  // namespace gvx
