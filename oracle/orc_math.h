/*
 * orc_math.h -- TEST INFRASTRUCTURE.  Small fp64 vector/quaternion helpers that
 * restate the Eigen 3.3 semantics the reference relies on
 * (common/rotation.h:72-119).  Quaternions are stored as
 * (x, y, z, w) exactly like Eigen's coeffs() and the reference's pose[3..6].
 * Every expression is evaluated left to right; no FMA contraction.
 */
#ifndef ORC_MATH_H
#define ORC_MATH_H

#include <math.h>
#include <string.h>

typedef struct {
    double x, y, z, w;
} oq;

static inline oq oq_make(double w, double x, double y, double z) {
    oq q = {x, y, z, w};
    return q;
}
static inline oq oq_from_xyzw(const double* c) {
    oq q = {c[0], c[1], c[2], c[3]};
    return q;
}
static inline void oq_to_xyzw(oq q, double* c) {
    c[0] = q.x;
    c[1] = q.y;
    c[2] = q.z;
    c[3] = q.w;
}
static inline oq oq_identity(void) { return oq_make(1, 0, 0, 0); }

/* Eigen quaternion product a*b */
static inline oq oq_mul(oq a, oq b) {
    oq r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}
static inline double oq_sqnorm(oq q) { return q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w; }
/* Quaternion::inverse(): conjugate / squaredNorm */
static inline oq oq_inverse(oq q) {
    double n2 = oq_sqnorm(q);
    oq r = {0, 0, 0, 0};
    if (n2 > 0) {
        r.x = -q.x / n2;
        r.y = -q.y / n2;
        r.z = -q.z / n2;
        r.w = q.w / n2;
    }
    return r;
}
/* normalize(): coeffs /= sqrt(squaredNorm) */
static inline oq oq_normalized(oq q) {
    double n2 = oq_sqnorm(q);
    if (n2 > 0) {
        double n = sqrt(n2);
        q.x /= n;
        q.y /= n;
        q.z /= n;
        q.w /= n;
    }
    return q;
}
static inline void v3_cross(const double* a, const double* b, double* r) {
    double t0 = a[1] * b[2] - a[2] * b[1];
    double t1 = a[2] * b[0] - a[0] * b[2];
    double t2 = a[0] * b[1] - a[1] * b[0];
    r[0] = t0;
    r[1] = t1;
    r[2] = t2;
}
/* q * v (Eigen _transformVector): uv = 2 (q.vec x v); v + w uv + q.vec x uv */
static inline void oq_rotate(oq q, const double* v, double* r) {
    double qv[3] = {q.x, q.y, q.z};
    double uv[3], t[3];
    v3_cross(qv, v, uv);
    uv[0] += uv[0];
    uv[1] += uv[1];
    uv[2] += uv[2];
    v3_cross(qv, uv, t);
    for (int i = 0; i < 3; i++) r[i] = v[i] + q.w * uv[i] + t[i];
}
/* toRotationMatrix(), row-major */
static inline void oq_to_rot(oq q, double* R) {
    double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
    double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1.0 - (tyy + tzz);
    R[1] = txy - twz;
    R[2] = txz + twy;
    R[3] = txy + twz;
    R[4] = 1.0 - (txx + tzz);
    R[5] = tyz - twx;
    R[6] = txz - twy;
    R[7] = tyz + twx;
    R[8] = 1.0 - (txx + tyy);
}
/* Rotation::rotvec2quaternion: AngleAxis(|r|, r.normalized()) */
static inline oq oq_from_rotvec(const double* r) {
    double n2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
    double angle = sqrt(n2);
    double ax[3] = {r[0], r[1], r[2]};
    if (n2 > 0) {
        double n = sqrt(n2);
        ax[0] /= n;
        ax[1] /= n;
        ax[2] /= n;
    }
    double ha = 0.5 * angle;
    double s = sin(ha);
    return oq_make(cos(ha), s * ax[0], s * ax[1], s * ax[2]);
}
/* Rotation::skewSymmetric, row-major */
static inline void skew3(const double* v, double* S) {
    S[0] = 0;
    S[1] = -v[2];
    S[2] = v[1];
    S[3] = v[2];
    S[4] = 0;
    S[5] = -v[0];
    S[6] = -v[1];
    S[7] = v[0];
    S[8] = 0;
}
/* r = A(3x3) * v */
static inline void m3v(const double* A, const double* v, double* r) {
    double t[3];
    for (int i = 0; i < 3; i++) t[i] = A[3 * i] * v[0] + A[3 * i + 1] * v[1] + A[3 * i + 2] * v[2];
    r[0] = t[0];
    r[1] = t[1];
    r[2] = t[2];
}
/* C = A(3x3) * B(3x3) */
static inline void m3m(const double* A, const double* B, double* C) {
    double t[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
    memcpy(C, t, sizeof(t));
}
static inline void m3t(const double* A, double* T) {
    double t[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) t[3 * i + j] = A[3 * j + i];
    memcpy(T, t, sizeof(t));
}
/* Rotation::quaternionleft(q).bottomRightCorner<3,3>() = w I + skew(vec) */
static inline void qleft_br(oq q, double* M) {
    double v[3] = {q.x, q.y, q.z}, S[9];
    skew3(v, S);
    for (int i = 0; i < 9; i++) M[i] = ((i % 4) == 0 ? q.w : 0.0) + S[i];
}
/* Rotation::quaternionright(p).bottomRightCorner<3,3>() = w I - skew(vec) */
static inline void qright_br(oq q, double* M) {
    double v[3] = {q.x, q.y, q.z}, S[9];
    skew3(v, S);
    for (int i = 0; i < 9; i++) M[i] = ((i % 4) == 0 ? q.w : 0.0) - S[i];
}
/* 4x4 left/right matrices in (w, x, y, z) order, row-major */
static inline void qleft4(oq q, double* M) {
    double v[3] = {q.x, q.y, q.z}, B[9];
    qleft_br(q, B);
    M[0] = q.w;
    M[1] = -v[0];
    M[2] = -v[1];
    M[3] = -v[2];
    for (int i = 0; i < 3; i++) {
        M[4 * (i + 1)] = v[i];
        for (int j = 0; j < 3; j++) M[4 * (i + 1) + 1 + j] = B[3 * i + j];
    }
}
static inline void qright4(oq q, double* M) {
    double v[3] = {q.x, q.y, q.z}, B[9];
    qright_br(q, B);
    M[0] = q.w;
    M[1] = -v[0];
    M[2] = -v[1];
    M[3] = -v[2];
    for (int i = 0; i < 3; i++) {
        M[4 * (i + 1)] = v[i];
        for (int j = 0; j < 3; j++) M[4 * (i + 1) + 1 + j] = B[3 * i + j];
    }
}

#endif
