/*
 * factors.c -- TEST INFRASTRUCTURE (parity oracle + CPU baseline), see gvx_oracle.h.
 *
 * Restates ReprojectionFactor::Evaluate (factors/reprojection_factor.h:61-161)
 * and PoseParameterization::Plus (factors/pose_parameterization.h:34-49) in
 * fp64, with Eigen's left-to-right product chains.
 */
#include <string.h>

#include "gvx_oracle.h"
#include "orc_math.h"
#include "orc_pool.h"

/* C(2x3) = A(2x3) * B(3x3) */
static void m23m33(const double* A, const double* B, double* C) {
    double t[6];
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 3; j++)
            t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
    memcpy(C, t, sizeof(t));
}
static void m23v(const double* A, const double* v, double* r) {
    double t0 = A[0] * v[0] + A[1] * v[1] + A[2] * v[2];
    double t1 = A[3] * v[0] + A[4] * v[1] + A[5] * v[2];
    r[0] = t0;
    r[1] = t1;
}
/* J(2x7 row-major) <- [reduce * L | reduce * R | 0] */
static void jac_2x7(const double* red, const double* L, const double* R, double* J) {
    double a[6], b[6];
    m23m33(red, L, a);
    m23m33(red, R, b);
    for (int i = 0; i < 2; i++) {
        for (int j = 0; j < 3; j++) {
            J[7 * i + j] = a[3 * i + j];
            J[7 * i + 3 + j] = b[3 * i + j];
        }
        J[7 * i + 6] = 0.0;
    }
}

void orc_reproj_eval(const orc_reproj_const* c, const double* const* params, double* residual,
                     double** jac) {
    const double* P0 = params[0];
    const double* P1 = params[1];
    const double* EX = params[2];
    oq q0 = oq_make(P0[6], P0[3], P0[4], P0[5]);
    oq q1 = oq_make(P1[6], P1[3], P1[4], P1[5]);
    oq qic = oq_make(EX[6], EX[3], EX[4], EX[5]);
    const double* p0 = P0;
    const double* p1 = P1;
    const double* tic = EX;
    double id0 = params[3][0];
    double td = params[4][0];
    double sq = 1.0 / c->std;
    /* sqrt_info_ = diag(1/std, 1/std) as a 2x2 matrix */
    double SI[4] = {sq, 0.0, 0.0, sq};

    double pts0td[3], pts1td[3], pc0[3], pb0[3], pn[3], pb1[3], pts1[3], t[3];
    for (int i = 0; i < 3; i++) {
        pts0td[i] = c->pts0[i] - (td - c->td0) * c->vel0[i];
        pts1td[i] = c->pts1[i] - (td - c->td1) * c->vel1[i];
    }
    for (int i = 0; i < 3; i++) pc0[i] = pts0td[i] / id0;
    oq_rotate(qic, pc0, t);
    for (int i = 0; i < 3; i++) pb0[i] = t[i] + tic[i];
    oq_rotate(q0, pb0, t);
    for (int i = 0; i < 3; i++) pn[i] = t[i] + p0[i];
    for (int i = 0; i < 3; i++) t[i] = pn[i] - p1[i];
    oq_rotate(oq_inverse(q1), t, pb1);
    for (int i = 0; i < 3; i++) t[i] = pb1[i] - tic[i];
    oq_rotate(oq_inverse(qic), t, pts1);
    double d1 = pts1[2];
    double e0 = pts1[0] / d1 - pts1td[0];
    double e1 = pts1[1] / d1 - pts1td[1];
    residual[0] = SI[0] * e0 + SI[1] * e1;
    residual[1] = SI[2] * e0 + SI[3] * e1;
    if (!jac) return;

    double cb0n[9], cnb1[9], cbc[9], R[9];
    oq_to_rot(q0, cb0n);
    oq_to_rot(q1, R);
    m3t(R, cnb1);
    oq_to_rot(qic, R);
    m3t(R, cbc);
    double red0[6] = {1.0 / d1, 0, -pts1[0] / (d1 * d1), 0, 1.0 / d1, -pts1[1] / (d1 * d1)};
    double red[6];
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 3; j++) red[3 * i + j] = SI[2 * i] * red0[j] + SI[2 * i + 1] * red0[3 + j];

    double A[9], B[9], C[9], S[9], ncbc[9];
    for (int i = 0; i < 9; i++) ncbc[i] = -cbc[i];
    if (jac[0]) {
        m3m(cbc, cnb1, A);
        m3m(ncbc, cnb1, B);
        m3m(B, cb0n, B);
        skew3(pb0, S);
        m3m(B, S, B);
        jac_2x7(red, A, B, jac[0]);
    }
    if (jac[1]) {
        m3m(ncbc, cnb1, A);
        skew3(pb1, S);
        m3m(cbc, S, B);
        jac_2x7(red, A, B, jac[1]);
    }
    if (jac[2]) {
        m3m(cnb1, cb0n, C);
        for (int i = 0; i < 9; i++) C[i] = C[i] - ((i % 4) == 0 ? 1.0 : 0.0);
        m3m(cbc, C, A);
        double tmp_r[9], cbcT[9];
        m3m(cbc, cnb1, tmp_r);
        m3m(tmp_r, cb0n, tmp_r);
        m3t(cbc, cbcT);
        m3m(tmp_r, cbcT, tmp_r);
        double ntr[9], S1[9], S2[9], S3[9], u[3], w[3];
        for (int i = 0; i < 9; i++) ntr[i] = -tmp_r[i];
        skew3(pc0, S);
        m3m(ntr, S, S1);
        m3v(tmp_r, pc0, u);
        skew3(u, S2);
        m3v(cb0n, tic, u);
        for (int i = 0; i < 3; i++) u[i] = u[i] + p0[i] - p1[i];
        m3v(cnb1, u, w);
        for (int i = 0; i < 3; i++) w[i] = w[i] - tic[i];
        m3v(cbc, w, u);
        skew3(u, S3);
        for (int i = 0; i < 9; i++) B[i] = S1[i] + S2[i] + S3[i];
        jac_2x7(red, A, B, jac[2]);
    }
    if (jac[3] || jac[4]) {
        double nred[6], M[6], cbcT[9], v[2];
        for (int i = 0; i < 6; i++) nred[i] = -red[i];
        m3t(cbc, cbcT);
        m23m33(nred, cbc, M);
        m23m33(M, cnb1, M);
        m23m33(M, cb0n, M);
        m23m33(M, cbcT, M);
        if (jac[3]) {
            m23v(M, pts0td, v);
            double dd = id0 * id0;
            jac[3][0] = v[0] / dd;
            jac[3][1] = v[1] / dd;
        }
        if (jac[4]) {
            m23v(M, c->vel0, v);
            double s0 = SI[0] * c->vel1[0] + SI[1] * c->vel1[1];
            double s1 = SI[2] * c->vel1[0] + SI[3] * c->vel1[1];
            jac[4][0] = v[0] / id0 + s0;
            jac[4][1] = v[1] / id0 + s1;
        }
    }
}

void orc_pose_plus(const double* x, const double* delta, double* xp) {
    oq q = oq_from_xyzw(x + 3);
    oq dq = oq_from_rotvec(delta + 3);
    for (int i = 0; i < 3; i++) xp[i] = x[i] + delta[i];
    oq r = oq_normalized(oq_mul(q, dq));
    oq_to_xyzw(r, xp + 3);
}

/* ------------------------------------------------------------------ batches */
typedef struct {
    const orc_reproj_const* c;
    const double* params;
    const int* offs;
    double *res, *jac;
} reproj_job;

static void reproj_range(void* ctx, int b, int e) {
    const reproj_job* j = (const reproj_job*)ctx;
    for (int i = b; i < e; ++i) {
        const int* o = j->offs + 5 * i;
        const double* prm[5] = {j->params + o[0], j->params + o[1], j->params + o[2], j->params + o[3],
                                j->params + o[4]};
        double* J = j->jac ? j->jac + 46 * (size_t)i : NULL;
        double* jb[5] = {J, J ? J + 14 : NULL, J ? J + 28 : NULL, J ? J + 42 : NULL, J ? J + 44 : NULL};
        orc_reproj_eval(j->c + i, prm, j->res + 2 * (size_t)i, J ? jb : NULL);
    }
}

void orc_reproj_eval_batch(int n, const orc_reproj_const* c, const double* params, const int* offs,
                           double* residuals, double* jacobians, int nthreads) {
    reproj_job j = {c, params, offs, residuals, jacobians};
    orc_parallel_for(n, nthreads, reproj_range, &j);
}

typedef struct {
    const orc_preint* const* segs;
    const double* params;
    const int* offs;
    double *res, *jac;
} preint_job;

static void preint_range(void* ctx, int b, int e) {
    const preint_job* j = (const preint_job*)ctx;
    for (int i = b; i < e; ++i) {
        const int* o = j->offs + 4 * i;
        const double* prm[4] = {j->params + o[0], j->params + o[1], j->params + o[2], j->params + o[3]};
        double* J = j->jac ? j->jac + 480 * (size_t)i : NULL;
        double* jb[4] = {J, J ? J + 105 : NULL, J ? J + 240 : NULL, J ? J + 345 : NULL};
        orc_preint_factor_eval(j->segs[i], prm, j->res + 15 * (size_t)i, J ? jb : NULL);
    }
}

void orc_preint_factor_eval_batch(int n, const orc_preint* const* segs, const double* params, const int* offs,
                                  double* residuals, double* jacobians, int nthreads) {
    preint_job j = {segs, params, offs, residuals, jacobians};
    orc_parallel_for(n, nthreads, preint_range, &j);
}
