/*
 * preint.c -- TEST INFRASTRUCTURE (parity oracle + CPU baseline), see gvx_oracle.h.
 *
 * Restates, sequentially and in fp64:
 *   PreintegrationBase           preintegration/preintegration_base.cc:25-125
 *   PreintegrationNormal         preintegration/preintegration_normal.cc:27-258
 *   PreintegrationEarth          preintegration/preintegration_earth.cc:26-338
 *   PreintegrationFactor         preintegration/preintegration_factor.h:45-69
 *   Earth::iewn(origin, local)   common/earth.h:158-237
 * Dense 15x15 products sum over k in ascending order; the inverse is a
 * partial-pivot LU (first max |a| pivot) with axpy-form substitutions, and the
 * Cholesky is Eigen's unblocked left-looking LLT.
 */
#include <stdlib.h>
#include <string.h>

#include "gvx_oracle.h"
#include "orc_math.h"

#define NS 15
#define NN 12

static const double WGS84_WIE = 7.2921151467E-5;
static const double WGS84_RA = 6378137.0000000000;
static const double WGS84_E1 = 0.0066943799901413156;

/* C(m x n) = A(m x k) * B(k x n), row-major, k ascending */
static void matmul(const double* A, const double* B, double* C, int m, int k, int n) {
    double* t = (double*)malloc(sizeof(double) * m * n);
    for (int i = 0; i < m; i++)
        for (int j = 0; j < n; j++) {
            double s = A[i * k] * B[j];
            for (int l = 1; l < k; l++) s = s + A[i * k + l] * B[l * n + j];
            t[i * n + j] = s;
        }
    memcpy(C, t, sizeof(double) * m * n);
    free(t);
}
static void transpose(const double* A, double* T, int m, int n) {
    for (int i = 0; i < m; i++)
        for (int j = 0; j < n; j++) T[j * m + i] = A[i * n + j];
}
static void set_block(double* M, int ld, int r, int c, const double* B3) {
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) M[(r + i) * ld + c + j] = B3[3 * i + j];
}
static void get_block(const double* M, int ld, int r, int c, double* B3) {
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) B3[3 * i + j] = M[(r + i) * ld + c + j];
}
static void diag3(double v, double* B) {
    memset(B, 0, sizeof(double) * 9);
    B[0] = B[4] = B[8] = v;
}

/* ---- Earth model (common/earth.h) ---- */
static double earth_rn(double lat) {
    double s = sin(lat);
    return WGS84_RA / sqrt(1.0 - WGS84_E1 * s * s);
}
void orc_earth_iewn(const double origin[3], const double local[3], double iewn[3]) {
    /* blh2ecef(origin) */
    double cl = cos(origin[0]), sl = sin(origin[0]), co = cos(origin[1]), so = sin(origin[1]);
    double rn = earth_rn(origin[0]), rnh = rn + origin[2];
    double e0[3] = {rnh * cl * co, rnh * cl * so, (rnh - rn * WGS84_E1) * sl};
    /* cne(origin) */
    double C[9] = {-sl * co, -so, -cl * co, -sl * so, co, -cl * so, cl, 0, -sl};
    double d[3];
    m3v(C, local, d);
    double e1[3] = {e0[0] + d[0], e0[1] + d[1], e0[2] + d[2]};
    /* ecef2blh */
    double p = sqrt(e1[0] * e1[0] + e1[1] * e1[1]);
    double lat = atan(e1[2] / (p * (1.0 - WGS84_E1)));
    double h = 0, h2;
    do {
        h2 = h;
        rn = earth_rn(lat);
        h = p / cos(lat) - rn;
        lat = atan(e1[2] / (p * (1.0 - WGS84_E1 * rn / (rn + h))));
    } while (fabs(h - h2) > 1.0e-4);
    iewn[0] = WGS84_WIE * cos(lat);
    iewn[1] = 0;
    iewn[2] = -WGS84_WIE * sin(lat);
}

/* ---- state handling ---- */
static void set_noise(orc_preint* s, const orc_imu_params* prm) {
    memset(s->noise, 0, sizeof(s->noise));
    double v[4] = {prm->gyr_arw * prm->gyr_arw, prm->acc_vrw * prm->acc_vrw,
                   2 * prm->gyr_bias_std * prm->gyr_bias_std / prm->corr_time,
                   2 * prm->acc_bias_std * prm->acc_bias_std / prm->corr_time};
    for (int b = 0; b < 4; b++)
        for (int i = 0; i < 3; i++) s->noise[(3 * b + i) * NN + 3 * b + i] = v[b];
}

/* resetState(state, NUM_STATE) of both variants */
static void reset_state(orc_preint* s, const orc_state* state, const double iewn[3]) {
    s->delta_time = 0;
    memset(&s->delta, 0, sizeof(s->delta));
    s->delta.q[3] = 1.0;
    memcpy(s->delta.bg, state->bg, sizeof(double) * 3);
    memcpy(s->delta.ba, state->ba, sizeof(double) * 3);
    memset(s->jacobian, 0, sizeof(s->jacobian));
    for (int i = 0; i < NS; i++) s->jacobian[i * NS + i] = 1.0;
    memset(s->covariance, 0, sizeof(s->covariance));
    if (s->variant == ORC_PREINT_EARTH) {
        memcpy(s->q0, s->current.q, sizeof(double) * 4);
        memcpy(s->iewn, iewn, sizeof(double) * 3);
    }
}

/* PreintegrationBase::compensationBias */
static void comp_bias(const orc_preint* s, const orc_imu* in, orc_imu* out) {
    *out = *in;
    for (int i = 0; i < 3; i++) {
        out->dtheta[i] = out->dtheta[i] - out->dt * s->delta.bg[i];
        out->dvel[i] = out->dvel[i] - out->dt * s->delta.ba[i];
    }
}

static void dvfb_of(const orc_imu* pre, const orc_imu* cur, double* dvfb) {
    double c1[3], c2[3], c3[3];
    v3_cross(cur->dtheta, cur->dvel, c1);
    v3_cross(pre->dtheta, cur->dvel, c2);
    v3_cross(pre->dvel, cur->dtheta, c3);
    for (int i = 0; i < 3; i++) dvfb[i] = cur->dvel[i] + 0.5 * c1[i] + 1.0 / 12.0 * (c2[i] + c3[i]);
}
static void dtheta_of(const orc_imu* pre, const orc_imu* cur, double* dth) {
    double c[3];
    v3_cross(pre->dtheta, cur->dtheta, c);
    for (int i = 0; i < 3; i++) dth[i] = cur->dtheta[i] + 1.0 / 12.0 * c[i];
}

/* PreintegrationBase::integration (normal variant state propagation) */
static void integration_normal(orc_preint* s, const orc_imu* pre, const orc_imu* cur) {
    double dt = cur->dt;
    s->delta_time += dt;
    s->end_time = cur->time;
    s->current.time = cur->time;
    double dvfb[3], R[9], dvel[3];
    dvfb_of(pre, cur, dvfb);
    oq_to_rot(oq_from_xyzw(s->current.q), R);
    m3v(R, dvfb, dvel);
    for (int i = 0; i < 3; i++) dvel[i] = dvel[i] + s->gravity[i] * dt;
    for (int i = 0; i < 3; i++) s->current.p[i] += dt * s->current.v[i] + 0.5 * dt * dvel[i];
    for (int i = 0; i < 3; i++) s->current.v[i] += dvel[i];
    double dth[3];
    dtheta_of(pre, cur, dth);
    oq dq = oq_from_rotvec(dth);
    oq q = oq_normalized(oq_mul(oq_from_xyzw(s->current.q), dq));
    oq_to_xyzw(q, s->current.q);
    oq_to_rot(oq_from_xyzw(s->delta.q), R);
    m3v(R, dvfb, dvel);
    for (int i = 0; i < 3; i++) s->delta.p[i] += dt * s->delta.v[i] + 0.5 * dt * dvel[i];
    for (int i = 0; i < 3; i++) s->delta.v[i] += dvel[i];
    q = oq_normalized(oq_mul(oq_from_xyzw(s->delta.q), dq));
    oq_to_xyzw(q, s->delta.q);
}

/* PreintegrationEarth::integrationProcess state part (preintegration_earth.cc:205-257) */
static void integration_earth(orc_preint* s, const orc_imu* pre, const orc_imu* cur, int step) {
    double dt = cur->dt;
    s->delta_time += dt;
    s->end_time = cur->time;
    s->current.time = cur->time;
    double dvfb[3], c[3], dvcg[3];
    dvfb_of(pre, cur, dvfb);
    v3_cross(s->iewn, s->current.v, c);
    for (int i = 0; i < 3; i++) dvcg[i] = (s->gravity[i] - 2.0 * c[i]) * dt;
    double dnn[3] = {-s->iewn[0] * dt, -s->iewn[1] * dt, -s->iewn[2] * dt};
    oq qnn = oq_from_rotvec(dnn);
    double Rnn[9], M1[9], Rq[9], dvel[3];
    oq_to_rot(qnn, Rnn);
    for (int i = 0; i < 9; i++) M1[i] = 0.5 * (((i % 4) == 0 ? 1.0 : 0.0) + Rnn[i]);
    oq_to_rot(oq_from_xyzw(s->current.q), Rq);
    m3m(M1, Rq, M1);
    m3v(M1, dvfb, dvel);
    for (int i = 0; i < 3; i++) dvel[i] = dvel[i] + dvcg[i];
    for (int i = 0; i < 3; i++) s->current.p[i] += dt * s->current.v[i] + 0.5 * dt * dvel[i];
    for (int i = 0; i < 3; i++) s->current.v[i] += dvel[i];
    s->pn[4 * step + 0] = dt;
    memcpy(&s->pn[4 * step + 1], s->current.p, sizeof(double) * 3);
    double dth[3];
    dtheta_of(pre, cur, dth);
    oq dq = oq_from_rotvec(dth);
    oq q = oq_normalized(oq_mul(oq_mul(qnn, oq_from_xyzw(s->current.q)), dq));
    oq_to_xyzw(q, s->current.q);
    double sc = -(s->delta_time - 0.5 * dt);
    double dnn2[3] = {sc * s->iewn[0], sc * s->iewn[1], sc * s->iewn[2]};
    oq q0 = oq_from_xyzw(s->q0);
    oq qm = oq_mul(oq_mul(oq_mul(oq_inverse(q0), oq_from_rotvec(dnn2)), q0), oq_from_xyzw(s->delta.q));
    double R[9];
    oq_to_rot(qm, R);
    m3v(R, dvfb, dvel);
    for (int i = 0; i < 3; i++) s->delta.p[i] += dt * s->delta.v[i] + 0.5 * dt * dvel[i];
    for (int i = 0; i < 3; i++) s->delta.v[i] += dvel[i];
    q = oq_normalized(oq_mul(oq_from_xyzw(s->delta.q), dq));
    oq_to_xyzw(q, s->delta.q);
}

/* updateJacobianAndCovariance of both variants */
static void update_jc(orc_preint* s, const orc_imu* cur, double corr_time) {
    double phi[NS * NS], gt[NS * NN], B[9], S[9], C[9];
    memset(phi, 0, sizeof(phi));
    memset(gt, 0, sizeof(gt));
    double dt = cur->dt;
    double cbb0[9]; /* Earth: cbb0; Normal: -R(delta q) */
    double gR[9];   /* gt(3:6,3:6) */
    double g60;     /* gt(6:9,0:3) diagonal */
    if (s->variant == ORC_PREINT_EARTH) {
        double dnn[3] = {-s->iewn[0] * s->delta_time, -s->iewn[1] * s->delta_time,
                         -s->iewn[2] * s->delta_time};
        oq q0 = oq_from_xyzw(s->q0);
        oq qm = oq_mul(oq_mul(oq_mul(oq_inverse(q0), oq_from_rotvec(dnn)), q0), oq_from_xyzw(s->delta.q));
        double R[9];
        oq_to_rot(qm, R);
        for (int i = 0; i < 9; i++) cbb0[i] = -R[i];
        memcpy(gR, cbb0, sizeof(gR));
        g60 = -1.0;
    } else {
        double R[9];
        oq_to_rot(oq_from_xyzw(s->delta.q), R);
        for (int i = 0; i < 9; i++) cbb0[i] = -R[i];
        memcpy(gR, R, sizeof(gR));
        g60 = 1.0;
    }
    diag3(1.0, B);
    set_block(phi, NS, 0, 0, B);
    diag3(dt, B);
    set_block(phi, NS, 0, 3, B);
    diag3(1.0, B);
    set_block(phi, NS, 3, 3, B);
    skew3(cur->dvel, S);
    m3m(cbb0, S, C);
    set_block(phi, NS, 3, 6, C);
    for (int i = 0; i < 9; i++) C[i] = cbb0[i] * dt;
    set_block(phi, NS, 3, 12, C);
    skew3(cur->dtheta, S);
    for (int i = 0; i < 9; i++) C[i] = ((i % 4) == 0 ? 1.0 : 0.0) - S[i];
    set_block(phi, NS, 6, 6, C);
    diag3(-dt, B);
    set_block(phi, NS, 6, 9, B);
    diag3(1 - dt / corr_time, B);
    set_block(phi, NS, 9, 9, B);
    set_block(phi, NS, 12, 12, B);

    matmul(phi, s->jacobian, s->jacobian, NS, NS, NS);

    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            gt[(3 + i) * NN + 3 + j] = gR[3 * i + j];
            gt[(6 + i) * NN + 0 + j] = i == j ? g60 : 0.0;
            gt[(9 + i) * NN + 6 + j] = i == j ? 1.0 : 0.0;
            gt[(12 + i) * NN + 9 + j] = i == j ? 1.0 : 0.0;
        }
    double gtT[NN * NS], phiT[NS * NS], t1[NS * NN], A[NS * NS], G[NS * NS], Bm[NS * NS], Qk[NS * NS];
    transpose(gt, gtT, NS, NN);
    transpose(phi, phiT, NS, NS);
    /* A = ((phi * gt) * noise) * gt^T */
    matmul(phi, gt, t1, NS, NS, NN);
    matmul(t1, s->noise, t1, NS, NN, NN);
    matmul(t1, gtT, A, NS, NN, NS);
    /* Bm = ((gt * noise) * gt^T) * phi^T */
    matmul(gt, s->noise, t1, NS, NN, NN);
    matmul(t1, gtT, G, NS, NN, NS);
    matmul(G, phiT, Bm, NS, NS, NS);
    for (int i = 0; i < NS * NS; i++) Qk[i] = 0.5 * dt * (A[i] + Bm[i]);
    /* P = (phi * P) * phi^T + Qk */
    matmul(phi, s->covariance, G, NS, NS, NS);
    matmul(G, phiT, G, NS, NS, NS);
    for (int i = 0; i < NS * NS; i++) s->covariance[i] = G[i] + Qk[i];
}

static void integration_process(orc_preint* s, const orc_imu* imu, int index, double corr_time) {
    orc_imu pre, cur;
    comp_bias(s, &imu[index - 1], &pre);
    comp_bias(s, &imu[index], &cur);
    if (s->variant == ORC_PREINT_EARTH)
        integration_earth(s, &pre, &cur, index - 1);
    else
        integration_normal(s, &pre, &cur);
    update_jc(s, &cur, corr_time);
}

void orc_preint_integrate(orc_preint* s, int variant, const orc_imu_params* prm, const orc_imu* imu,
                          int m, const orc_state* state0, const double iewn[3]) {
    memset(s, 0, sizeof(*s));
    s->variant = variant;
    s->m = m;
    s->current = *state0;
    s->start_time = imu[0].time;
    s->end_time = imu[0].time;
    s->gravity[0] = 0;
    s->gravity[1] = 0;
    s->gravity[2] = prm->gravity;
    s->pn = (double*)calloc((size_t)4 * (m > 1 ? m - 1 : 1), sizeof(double));
    reset_state(s, state0, iewn);
    set_noise(s, prm);
    for (int k = 1; k < m; k++) integration_process(s, imu, k, prm->corr_time);
}

void orc_preint_reintegrate(orc_preint* s, const orc_imu_params* prm, const orc_imu* imu,
                            const orc_state* state, const double iewn[3]) {
    s->current = *state;
    reset_state(s, state, iewn);
    for (int k = 1; k < s->m; k++) integration_process(s, imu, k, prm->corr_time);
}

void orc_preint_free(orc_preint* s) {
    free(s->pn);
    s->pn = NULL;
}

/* ---- evaluate: sqrt_information_ = LLT(P^-1).matrixL().transpose() ---- */

/* PartialPivLU inverse: unblocked LU (rank-1 updates), then P*I, unit-lower
   forward substitution and upper back substitution, both in axpy order. */
static void lu_inverse(const double* P, double* inv) {
    double a[NS * NS];
    int perm[NS];
    memcpy(a, P, sizeof(a));
    for (int i = 0; i < NS; i++) perm[i] = i;
    for (int k = 0; k < NS; k++) {
        int piv = k;
        double best = fabs(a[k * NS + k]);
        for (int i = k + 1; i < NS; i++)
            if (fabs(a[i * NS + k]) > best) {
                best = fabs(a[i * NS + k]);
                piv = i;
            }
        if (piv != k) {
            for (int j = 0; j < NS; j++) {
                double t = a[k * NS + j];
                a[k * NS + j] = a[piv * NS + j];
                a[piv * NS + j] = t;
            }
            int t = perm[k];
            perm[k] = perm[piv];
            perm[piv] = t;
        }
        if (a[k * NS + k] != 0.0)
            for (int i = k + 1; i < NS; i++) a[i * NS + k] = a[i * NS + k] / a[k * NS + k];
        for (int i = k + 1; i < NS; i++)
            for (int j = k + 1; j < NS; j++) a[i * NS + j] = a[i * NS + j] - a[i * NS + k] * a[k * NS + j];
    }
    /* X = P * I: row i of X is e_{perm[i]} */
    double x[NS * NS];
    memset(x, 0, sizeof(x));
    for (int i = 0; i < NS; i++) x[i * NS + perm[i]] = 1.0;
    for (int k = 0; k < NS; k++)
        for (int i = k + 1; i < NS; i++)
            for (int c = 0; c < NS; c++) x[i * NS + c] = x[i * NS + c] - a[i * NS + k] * x[k * NS + c];
    for (int k = NS - 1; k >= 0; k--) {
        for (int c = 0; c < NS; c++) x[k * NS + c] = x[k * NS + c] / a[k * NS + k];
        for (int i = 0; i < k; i++)
            for (int c = 0; c < NS; c++) x[i * NS + c] = x[i * NS + c] - a[i * NS + k] * x[k * NS + c];
    }
    memcpy(inv, x, sizeof(x));
}

/* Eigen llt_inplace<Lower>::unblocked on the lower triangle; returns L^T. */
static void llt_upper(const double* A, double* U) {
    double L[NS * NS];
    memcpy(L, A, sizeof(L));
    for (int k = 0; k < NS; k++) {
        double x = L[k * NS + k];
        if (k > 0) {
            double sq = 0;
            for (int j = 0; j < k; j++) sq = sq + L[k * NS + j] * L[k * NS + j];
            x = x - sq;
        }
        x = sqrt(x);
        L[k * NS + k] = x;
        for (int i = k + 1; i < NS; i++) {
            if (k > 0) {
                double d = 0;
                for (int j = 0; j < k; j++) d = d + L[i * NS + j] * L[k * NS + j];
                L[i * NS + k] = L[i * NS + k] - d;
            }
            L[i * NS + k] = L[i * NS + k] / x;
        }
    }
    for (int i = 0; i < NS; i++)
        for (int j = 0; j < NS; j++) U[i * NS + j] = j >= i ? L[j * NS + i] : 0.0;
}

void orc_preint_factor_eval(const orc_preint* s, const double* const* params, double* residual,
                            double** jac) {
    /* constructState (preintegration_earth.cc:186-203) */
    const double *ps0 = params[0], *m0 = params[1], *ps1 = params[2], *m1 = params[3];
    oq q0 = oq_make(ps0[6], ps0[3], ps0[4], ps0[5]);
    oq q1 = oq_make(ps1[6], ps1[3], ps1[4], ps1[5]);
    const double *p0 = ps0, *p1 = ps1, *v0 = m0, *v1 = m1;
    const double *bg0 = m0 + 3, *ba0 = m0 + 6, *bg1 = m1 + 3, *ba1 = m1 + 6;
    const double dtt = s->delta_time;

    double inv[NS * NS], sqi[NS * NS];
    lu_inverse(s->covariance, inv);
    llt_upper(inv, sqi);

    double dp_dbg[9], dp_dba[9], dv_dbg[9], dv_dba[9], dq_dbg[9];
    get_block(s->jacobian, NS, 0, 9, dp_dbg);
    get_block(s->jacobian, NS, 0, 12, dp_dba);
    get_block(s->jacobian, NS, 3, 9, dv_dbg);
    get_block(s->jacobian, NS, 3, 12, dv_dba);
    get_block(s->jacobian, NS, 6, 9, dq_dbg);
    double dbg[3], dba[3], t[3], u[3];
    for (int i = 0; i < 3; i++) {
        dbg[i] = bg0[i] - s->delta.bg[i];
        dba[i] = ba0[i] - s->delta.ba[i];
    }
    double cp[3], cv[3];
    m3v(dp_dba, dba, t);
    m3v(dp_dbg, dbg, u);
    for (int i = 0; i < 3; i++) cp[i] = s->delta.p[i] + t[i] + u[i];
    m3v(dv_dba, dba, t);
    m3v(dv_dbg, dbg, u);
    for (int i = 0; i < 3; i++) cv[i] = s->delta.v[i] + t[i] + u[i];
    m3v(dq_dbg, dbg, t);
    oq cq = oq_mul(oq_from_xyzw(s->delta.q), oq_from_rotvec(t));

    double r[NS];
    const double* g = s->gravity;
    double J0[NS * 7], J1[NS * 9], J2[NS * 7], J3[NS * 9];
    memset(J0, 0, sizeof(J0));
    memset(J1, 0, sizeof(J1));
    memset(J2, 0, sizeof(J2));
    memset(J3, 0, sizeof(J3));
    oq q0i = oq_inverse(q0);
    double cnb0[9];
    oq_to_rot(q0i, cnb0);
    double M[9], N[9], L4[16], R4[16], P4[16];

    if (s->variant == ORC_PREINT_EARTH) {
        double S[9], S2[9];
        skew3(s->iewn, S);
        double pc[3] = {0, 0, 0};
        for (int k = 0; k < s->m - 1; k++)
            for (int i = 0; i < 3; i++) pc[i] = pc[i] + (s->pn[4 * k + 1 + i] - p0[i]) * s->pn[4 * k];
        for (int i = 0; i < 9; i++) S2[i] = 2.0 * S[i];
        m3v(S2, pc, pc);
        double dp[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]}, vc[3];
        m3v(S2, dp, vc);
        double dnn[3] = {-s->iewn[0] * dtt, -s->iewn[1] * dtt, -s->iewn[2] * dtt};
        oq qnn = oq_from_rotvec(dnn);
        double dpn[3], dvn[3];
        for (int i = 0; i < 3; i++) {
            dpn[i] = p1[i] - p0[i] - v0[i] * dtt - 0.5 * g[i] * dtt * dtt + pc[i];
            dvn[i] = v1[i] - v0[i] - g[i] * dtt + vc[i];
        }
        oq qb0b1 = oq_mul(oq_mul(oq_inverse(q1), qnn), q0);
        m3v(cnb0, dpn, t);
        for (int i = 0; i < 3; i++) r[i] = t[i] - cp[i];
        m3v(cnb0, dvn, t);
        for (int i = 0; i < 3; i++) r[3 + i] = t[i] - cv[i];
        oq e = oq_mul(qb0b1, cq);
        r[6] = 2 * e.x;
        r[7] = 2 * e.y;
        r[8] = 2 * e.z;
        if (jac) {
            /* Pose0 */
            double C2[9];
            for (int i = 0; i < 9; i++) C2[i] = 2.0 * cnb0[i];
            m3m(C2, S, M);
            for (int i = 0; i < 9; i++) N[i] = -cnb0[i] - M[i] * dtt;
            set_block(J0, 7, 0, 0, N);
            m3v(cnb0, dpn, t);
            skew3(t, N);
            set_block(J0, 7, 0, 3, N);
            for (int i = 0; i < 9; i++) C2[i] = -2.0 * cnb0[i];
            m3m(C2, S, N);
            set_block(J0, 7, 3, 0, N);
            m3v(cnb0, dvn, t);
            skew3(t, N);
            set_block(J0, 7, 3, 3, N);
            qleft4(qb0b1, L4);
            qright4(cq, R4);
            matmul(L4, R4, P4, 4, 4, 4);
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) N[3 * i + j] = P4[4 * (i + 1) + j + 1];
            set_block(J0, 7, 6, 3, N);
            /* Pose1 */
            set_block(J2, 7, 0, 0, cnb0);
            for (int i = 0; i < 9; i++) C2[i] = 2.0 * cnb0[i];
            m3m(C2, S, N);
            set_block(J2, 7, 3, 0, N);
            qright_br(oq_mul(qb0b1, cq), N);
            for (int i = 0; i < 9; i++) N[i] = -N[i];
            set_block(J2, 7, 6, 3, N);
            /* Mix0 */
            for (int i = 0; i < 9; i++) N[i] = -cnb0[i] * dtt;
            set_block(J1, 9, 0, 0, N);
            for (int i = 0; i < 9; i++) N[i] = -dp_dbg[i];
            set_block(J1, 9, 0, 3, N);
            for (int i = 0; i < 9; i++) N[i] = -dp_dba[i];
            set_block(J1, 9, 0, 6, N);
            for (int i = 0; i < 9; i++) N[i] = -cnb0[i];
            set_block(J1, 9, 3, 0, N);
            for (int i = 0; i < 9; i++) N[i] = -dv_dbg[i];
            set_block(J1, 9, 3, 3, N);
            for (int i = 0; i < 9; i++) N[i] = -dv_dba[i];
            set_block(J1, 9, 3, 6, N);
            qleft_br(oq_mul(qb0b1, oq_from_xyzw(s->delta.q)), M);
            m3m(M, dq_dbg, N);
            set_block(J1, 9, 6, 3, N);
        }
    } else {
        double dp[3], dv[3], rp[3], rv[3];
        for (int i = 0; i < 3; i++) {
            dp[i] = p1[i] - p0[i] - v0[i] * dtt - 0.5 * g[i] * dtt * dtt;
            dv[i] = v1[i] - v0[i] - g[i] * dtt;
        }
        oq_rotate(q0i, dp, rp);
        oq_rotate(q0i, dv, rv);
        for (int i = 0; i < 3; i++) {
            r[i] = rp[i] - cp[i];
            r[3 + i] = rv[i] - cv[i];
        }
        oq e = oq_mul(oq_mul(oq_inverse(cq), q0i), q1);
        r[6] = 2 * e.x;
        r[7] = 2 * e.y;
        r[8] = 2 * e.z;
        if (jac) {
            for (int i = 0; i < 9; i++) N[i] = -cnb0[i];
            set_block(J0, 7, 0, 0, N);
            skew3(rp, N);
            set_block(J0, 7, 0, 3, N);
            skew3(rv, N);
            set_block(J0, 7, 3, 3, N);
            qleft4(oq_mul(oq_inverse(q1), q0), L4);
            qright4(cq, R4);
            matmul(L4, R4, P4, 4, 4, 4);
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) N[3 * i + j] = -P4[4 * (i + 1) + j + 1];
            set_block(J0, 7, 6, 3, N);
            set_block(J2, 7, 0, 0, cnb0);
            qleft_br(e, N);
            set_block(J2, 7, 6, 3, N);
            for (int i = 0; i < 9; i++) N[i] = -cnb0[i] * dtt;
            set_block(J1, 9, 0, 0, N);
            for (int i = 0; i < 9; i++) N[i] = -dp_dbg[i];
            set_block(J1, 9, 0, 3, N);
            for (int i = 0; i < 9; i++) N[i] = -dp_dba[i];
            set_block(J1, 9, 0, 6, N);
            for (int i = 0; i < 9; i++) N[i] = -cnb0[i];
            set_block(J1, 9, 3, 0, N);
            for (int i = 0; i < 9; i++) N[i] = -dv_dbg[i];
            set_block(J1, 9, 3, 3, N);
            for (int i = 0; i < 9; i++) N[i] = -dv_dba[i];
            set_block(J1, 9, 3, 6, N);
            qleft_br(oq_mul(oq_mul(oq_inverse(q1), q0), oq_from_xyzw(s->delta.q)), M);
            for (int i = 0; i < 9; i++) M[i] = -M[i];
            m3m(M, dq_dbg, N);
            set_block(J1, 9, 6, 3, N);
        }
    }
    for (int i = 0; i < 3; i++) {
        r[9 + i] = bg1[i] - bg0[i];
        r[12 + i] = ba1[i] - ba0[i];
    }
    double rr[NS];
    matmul(sqi, r, rr, NS, NS, 1);
    memcpy(residual, rr, sizeof(rr));
    if (!jac) return;
    /* common blocks of Mix0 / Mix1 */
    for (int i = 0; i < 3; i++) {
        J1[(9 + i) * 9 + 3 + i] = -1.0;
        J1[(12 + i) * 9 + 6 + i] = -1.0;
        J3[(9 + i) * 9 + 3 + i] = 1.0;
        J3[(12 + i) * 9 + 6 + i] = 1.0;
    }
    set_block(J3, 9, 3, 0, cnb0);
    if (jac[0]) matmul(sqi, J0, jac[0], NS, NS, 7);
    if (jac[1]) matmul(sqi, J1, jac[1], NS, NS, 9);
    if (jac[2]) matmul(sqi, J2, jac[2], NS, NS, 7);
    if (jac[3]) matmul(sqi, J3, jac[3], NS, NS, 9);
}
