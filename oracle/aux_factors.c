/*
 * aux_factors.c -- CPU restatement of the remaining Ceres cost functions of the
 * sliding window (TEST INFRASTRUCTURE ONLY; see gvx_oracle.h).  Paths relative
 * to /root/reference/ic_gvins/ic_gvins/.
 *
 *   orc_small_factor_eval  one of
 *     GNSS        GnssFactor::Evaluate (factors/gnss_factor.h:52-95)
 *     IMU_ERROR   ImuErrorFactor::Evaluate, NORMAL / EARTH options
 *                 (preintegration/imu_error_factor.h:45-66)
 *     POSE_PRIOR  ImuPosePriorFactor::Evaluate (preintegration/imu_pose_prior_factor.h:42-68)
 *     MIX_PRIOR   ImuMixPriorFactor::Evaluate, NORMAL / EARTH options
 *                 (preintegration/imu_mix_prior_factor.h:40-56)
 *   orc_marg_factor_eval   MarginalizationFactor::Evaluate
 *                          (factors/marginalization_factor.h:54-110)
 *
 * The sqrt_info matrices are diagonal: in sqrt_info * v every off-diagonal term
 * is an exact +-0 that leaves the sum unchanged, so the product is
 * sqrt_info(i,i) * v(i) with sqrt_info(i,i) = 1.0 / std(i), as written here.
 * The marginalisation residual e0 + J0 dx sums J0's columns in order; Eigen's
 * GEMV may reassociate that sum, so the tests hold it to a relative bound, not
 * bit for bit.  Parity unpinned against the reference binaries (Eigen and Ceres
 * absent); pinned by closed forms and numeric Jacobians in
 * tests/test_oracle_aux.py.
 */
#include <stdlib.h>
#include <string.h>

#include "gvx_oracle.h"
#include "orc_math.h"

/* ImuErrorFactor's constants (imu_error_factor.h:89-90), evaluated in the
   same order as the reference's constexpr initialisers */
#define ORC_PI 3.14159265358979323846
static const double IMU_GRY_BIAS_STD = 7200 / 3600.0 * ORC_PI / 180.0; /* 7200 deg / hr */
static const double IMU_ACC_BIAS_STD = 2.0e4 * 1.0e-5;                  /* 20000 mGal */

const int orc_small_factor_dims[4][3] = {
    /* residuals, parameter block size, constants per factor */
    {3, 7, 9},   /* GNSS: blh[3], std[3], lever[3] */
    {6, 9, 0},   /* IMU_ERROR */
    {6, 7, 13},  /* POSE_PRIOR: pose[7], std[6] */
    {9, 9, 18},  /* MIX_PRIOR: mix[9], std[9] */
};

static void gnss(const double* c, const double* p, double* res, double* jac) {
    const double *blh = c, *std = c + 3, *lever = c + 6;
    const oq q = oq_make(p[6], p[3], p[4], p[5]);
    double R[9], Rl[3], s[3];
    oq_to_rot(q, R);
    m3v(R, lever, Rl);
    for (int i = 0; i < 3; i++) s[i] = 1.0 / std[i];
    for (int i = 0; i < 3; i++) res[i] = s[i] * (p[i] + Rl[i] - blh[i]);
    if (!jac) return;
    double nR[9], S[9], B[9];
    for (int i = 0; i < 9; i++) nR[i] = -R[i];
    skew3(lever, S);
    m3m(nR, S, B); /* -q.toRotationMatrix() * skewSymmetric(lever) */
    memset(jac, 0, sizeof(double) * 21);
    for (int i = 0; i < 3; i++) {
        jac[i * 7 + i] = s[i] * 1.0;
        for (int j = 0; j < 3; j++) jac[i * 7 + 3 + j] = s[i] * B[i * 3 + j];
    }
}

static void imu_error(const double* p, double* res, double* jac) {
    for (int k = 0; k < 3; k++) {
        res[k] = p[k + 3] / IMU_GRY_BIAS_STD;
        res[k + 3] = p[k + 6] / IMU_ACC_BIAS_STD;
    }
    if (!jac) return;
    memset(jac, 0, sizeof(double) * 54);
    for (int k = 0; k < 3; k++) {
        jac[k * 9 + k + 3] = 1.0 / IMU_GRY_BIAS_STD;
        jac[(k + 3) * 9 + k + 6] = 1.0 / IMU_ACC_BIAS_STD;
    }
}

static void pose_prior(const double* c, const double* p, double* res, double* jac) {
    const double *prior = c, *std = c + 7;
    double r[6], s[6];
    for (int k = 0; k < 3; k++) r[k] = p[k] - prior[k];
    const oq qp = oq_make(prior[6], prior[3], prior[4], prior[5]);
    const oq q = oq_make(p[6], p[3], p[4], p[5]);
    const oq d = oq_mul(oq_inverse(q), qp);
    r[3] = 2 * d.x;
    r[4] = 2 * d.y;
    r[5] = 2 * d.z;
    for (int k = 0; k < 6; k++) s[k] = 1.0 / std[k];
    for (int k = 0; k < 6; k++) res[k] = s[k] * r[k];
    if (!jac) return;
    double M[9];
    qright_br(d, M);
    memset(jac, 0, sizeof(double) * 42);
    for (int k = 0; k < 3; k++) jac[k * 7 + k] = s[k] * 1.0;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) jac[(3 + i) * 7 + 3 + j] = s[3 + i] * -M[i * 3 + j];
}

static void mix_prior(const double* c, const double* p, double* res, double* jac) {
    const double *prior = c, *std = c + 9;
    for (int k = 0; k < 9; k++) res[k] = (p[k] - prior[k]) / std[k];
    if (!jac) return;
    memset(jac, 0, sizeof(double) * 81);
    for (int k = 0; k < 9; k++) jac[k * 9 + k] = 1.0 / std[k];
}

int orc_small_factor_eval(int kind, int n, const double* consts, const double* params, const int* offs,
                          double* residuals, double* jacobians) {
    if (kind < 0 || kind > 3) return -1;
    const int R = orc_small_factor_dims[kind][0], P = orc_small_factor_dims[kind][1],
              NC = orc_small_factor_dims[kind][2];
    for (int i = 0; i < n; i++) {
        const double* c = consts + (long)i * NC;
        const double* p = params + offs[i];
        double* res = residuals + (long)i * R;
        double* jac = jacobians ? jacobians + (long)i * R * P : 0;
        switch (kind) {
            case 0: gnss(c, p, res, jac); break;
            case 1: imu_error(p, res, jac); break;
            case 2: pose_prior(c, p, res, jac); break;
            default: mix_prior(c, p, res, jac); break;
        }
    }
    return 0;
}

void orc_marg_factor_eval(int r, int nb, const int* size, const int* index, const int* xoff, const double* x0,
                          const double* params, const double* J0, const double* e0, double* residuals,
                          double* jacobians) {
    double* dx = (double*)malloc(sizeof(double) * (r > 0 ? r : 1));
    for (int b = 0; b < nb; b++) {
        const double* x = params + xoff[b];
        const double* z = x0 + xoff[b];
        const int id = index[b];
        if (size[b] == 7) { /* POSE_GLOBAL_SIZE */
            const oq dq = oq_mul(oq_inverse(oq_make(z[6], z[3], z[4], z[5])), oq_make(x[6], x[3], x[4], x[5]));
            for (int k = 0; k < 3; k++) dx[id + k] = x[k] - z[k];
            const double s = dq.w < 0 ? -2.0 : 2.0;
            dx[id + 3] = s * dq.x;
            dx[id + 4] = s * dq.y;
            dx[id + 5] = s * dq.z;
        } else {
            for (int k = 0; k < size[b]; k++) dx[id + k] = x[k] - z[k];
        }
    }
    for (int i = 0; i < r; i++) {
        double acc = 0.0;
        for (int j = 0; j < r; j++) acc += J0[(long)j * r + i] * dx[j];
        residuals[i] = e0[i] + acc;
    }
    free(dx);
    if (!jacobians) return;
    for (int b = 0; b < nb; b++) {
        const int sz = size[b], local = sz == 7 ? 6 : sz;
        double* J = jacobians + (long)r * xoff[b];
        for (int i = 0; i < r; i++)
            for (int c = 0; c < sz; c++) J[i * sz + c] = c < local ? J0[(long)(index[b] + c) * r + i] : 0.0;
    }
}
