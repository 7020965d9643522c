// dmath.h -- fp64 device helpers with Eigen 3.3 evaluation order (quaternions
// stored x,y,z,w like Eigen coeffs() and the reference's pose[3..6];
// common/rotation.h:72-119).  Built with -ffp-contract=off: no FMA contraction.
#pragma once

#include <hip/hip_runtime.h>

namespace gvx {

struct dq {
    double x, y, z, w;
};

__device__ __forceinline__ dq dq_make(double w, double x, double y, double z) { return dq{x, y, z, w}; }
__device__ __forceinline__ dq dq_load(const double* c) { return dq{c[0], c[1], c[2], c[3]}; }
__device__ __forceinline__ void dq_store(dq q, double* c) {
    c[0] = q.x;
    c[1] = q.y;
    c[2] = q.z;
    c[3] = q.w;
}
// Eigen quaternion product a * b
__device__ __forceinline__ dq dq_mul(dq a, dq b) {
    dq r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}
__device__ __forceinline__ double dq_sqnorm(dq q) { return q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w; }
__device__ __forceinline__ dq dq_inv(dq q) {
    const double n2 = dq_sqnorm(q);
    if (n2 > 0) return dq{-q.x / n2, -q.y / n2, -q.z / n2, q.w / n2};
    return dq{0, 0, 0, 0};
}
__device__ __forceinline__ dq dq_normalized(dq q) {
    const double n2 = dq_sqnorm(q);
    if (n2 > 0) {
        const double n = sqrt(n2);
        q.x /= n;
        q.y /= n;
        q.z /= n;
        q.w /= n;
    }
    return q;
}
__device__ __forceinline__ void cross3(const double* a, const double* b, double* r) {
    const double t0 = a[1] * b[2] - a[2] * b[1];
    const double t1 = a[2] * b[0] - a[0] * b[2];
    const double t2 = a[0] * b[1] - a[1] * b[0];
    r[0] = t0;
    r[1] = t1;
    r[2] = t2;
}
// q * v (Eigen _transformVector)
__device__ __forceinline__ void dq_rotate(dq q, const double* v, double* r) {
    const double qv[3] = {q.x, q.y, q.z};
    double uv[3], t[3];
    cross3(qv, v, uv);
    uv[0] += uv[0];
    uv[1] += uv[1];
    uv[2] += uv[2];
    cross3(qv, uv, t);
    for (int i = 0; i < 3; ++i) r[i] = v[i] + q.w * uv[i] + t[i];
}
// toRotationMatrix, row-major
__device__ __forceinline__ void dq_rot(dq q, double* R) {
    const double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
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
// Rotation::rotvec2quaternion = AngleAxis(|r|, r.normalized())
__device__ __forceinline__ dq dq_from_rotvec(const double* r) {
    const double n2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
    const double angle = sqrt(n2);
    double ax[3] = {r[0], r[1], r[2]};
    if (n2 > 0) {
        const double n = sqrt(n2);
        ax[0] /= n;
        ax[1] /= n;
        ax[2] /= n;
    }
    const double ha = 0.5 * angle;
    const double s = sin(ha);
    return dq_make(cos(ha), s * ax[0], s * ax[1], s * ax[2]);
}
__device__ __forceinline__ void skew(const double* v, double* S) {
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
__device__ __forceinline__ void mv3(const double* A, const double* v, double* r) {
    double t[3];
    for (int i = 0; i < 3; ++i) t[i] = A[3 * i] * v[0] + A[3 * i + 1] * v[1] + A[3 * i + 2] * v[2];
    r[0] = t[0];
    r[1] = t[1];
    r[2] = t[2];
}
__device__ __forceinline__ void mm3(const double* A, const double* B, double* C) {
    double t[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
    for (int k = 0; k < 9; ++k) C[k] = t[k];
}
__device__ __forceinline__ void mt3(const double* A, double* T) {
    double t[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) t[3 * i + j] = A[3 * j + i];
    for (int k = 0; k < 9; ++k) T[k] = t[k];
}
// quaternionleft(q).bottomRightCorner<3,3>() = w I + [v]x ; right: w I - [v]x
__device__ __forceinline__ void qleft_br(dq q, double* M) {
    const double v[3] = {q.x, q.y, q.z};
    double S[9];
    skew(v, S);
    for (int i = 0; i < 9; ++i) M[i] = ((i % 4) == 0 ? q.w : 0.0) + S[i];
}
__device__ __forceinline__ void qright_br(dq q, double* M) {
    const double v[3] = {q.x, q.y, q.z};
    double S[9];
    skew(v, S);
    for (int i = 0; i < 9; ++i) M[i] = ((i % 4) == 0 ? q.w : 0.0) - S[i];
}
// (quaternionleft(a) * quaternionright(b)).bottomRightCorner<3,3>() of the 4x4
// product, k = 0..3 summed in order: entry (1+i, 1+j) = L[1+i][0]*R[0][1+j] + sum_k L[1+i][1+k] R[1+k][1+j]
__device__ __forceinline__ void qlr_br(dq a, dq b, double* M) {
    const double av[3] = {a.x, a.y, a.z}, bv[3] = {b.x, b.y, b.z};
    double L[9], R[9];
    qleft_br(a, L);
    qright_br(b, R);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            M[3 * i + j] = av[i] * -bv[j] + L[3 * i] * R[j] + L[3 * i + 1] * R[3 + j] + L[3 * i + 2] * R[6 + j];
}

// sqrt_information_ = LLT(covariance_.inverse()).matrixL().transpose() of one
// 15 x 15 covariance by a 16-lane group (lane gl) of a one-wave workgroup
// (preintegration_earth.cc:39-40; factors.hip sqrt_info_kernel and the
// covariance pass preint.hip preint_cov16_kernel share it): partial-pivot LU,
// axpy-form substitutions for the inverse and the left-looking unblocked LLT,
// each entry updated in the same k order as the sequential CPU restatement
// (oracle/preint.c).  Lane gl owns column k+1+gl of the LU's trailing block,
// column gl of the inverse (held in registers through both substitutions: a
// column depends only on itself and on A) and row gl in the LLT.  A (the
// covariance, row-major, on entry), X and perm are the group's LDS scratch;
// the result is stored upper triangular (sqrt_info[i][j] = L[j][i]) to dst
// unless dst is null.
constexpr int SI_N = 15;
__device__ __forceinline__ void sqrt_info_group(double* A, double* X, int* perm, int gl, double* dst) {
    if (gl < SI_N) perm[gl] = gl;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SI_N; ++k) {
        int piv = k;
        double best = fabs(A[k * SI_N + k]);
        for (int i = k + 1; i < SI_N; ++i) {
            const double v = fabs(A[i * SI_N + k]);
            if (v > best) {
                best = v;
                piv = i;
            }
        }
        __syncthreads();
        if (piv != k) {
            if (gl < SI_N) {
                const double t = A[k * SI_N + gl];
                A[k * SI_N + gl] = A[piv * SI_N + gl];
                A[piv * SI_N + gl] = t;
            }
            if (gl == 0) {
                const int t = perm[k];
                perm[k] = perm[piv];
                perm[piv] = t;
            }
        }
        __syncthreads();
        const double akk = A[k * SI_N + k];
        if (akk != 0.0 && gl > k && gl < SI_N) A[gl * SI_N + k] = A[gl * SI_N + k] / akk;
        __syncthreads();
        const int j = k + 1 + gl;  // trailing block column of this lane
        if (j < SI_N) {
            // every operand read before the first store (the rows are independent)
            double l[SI_N], u[SI_N];
            const double akj = A[k * SI_N + j];
#pragma unroll
            for (int i = k + 1; i < SI_N; ++i) {
                l[i] = A[i * SI_N + k];
                u[i] = A[i * SI_N + j];
            }
#pragma unroll
            for (int i = k + 1; i < SI_N; ++i) A[i * SI_N + j] = u[i] - l[i] * akj;
        }
        __syncthreads();
    }
    // inverse from the LU: X = P, then L^-1 and U^-1 column by column (lane gl:
    // column gl; a column's entries depend only on that column and on A)
    // (the column in registers: A is read-only here, so its reads issue early)
    if (gl < SI_N) {
        const int c = gl;
        double xc[SI_N];
#pragma unroll
        for (int i = 0; i < SI_N; ++i) xc[i] = perm[i] == c ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < SI_N; ++k)
#pragma unroll
            for (int i = k + 1; i < SI_N; ++i) xc[i] = xc[i] - A[i * SI_N + k] * xc[k];
#pragma unroll
        for (int k = SI_N - 1; k >= 0; --k) {
            xc[k] = xc[k] / A[k * SI_N + k];
#pragma unroll
            for (int i = 0; i < k; ++i) xc[i] = xc[i] - A[i * SI_N + k] * xc[k];
        }
#pragma unroll
        for (int i = 0; i < SI_N; ++i) X[i * SI_N + c] = xc[i];
    }
    __syncthreads();
    // Eigen llt_inplace<Lower>::unblocked on the lower triangle of X
#pragma unroll
    for (int k = 0; k < SI_N; ++k) {
        double x = X[k * SI_N + k];
        if (k > 0) {
            double sq = 0;
            for (int j = 0; j < k; ++j) sq = sq + X[k * SI_N + j] * X[k * SI_N + j];
            x = x - sq;
        }
        x = sqrt(x);
        __syncthreads();
        if (gl == 0) X[k * SI_N + k] = x;
        if (gl > k && gl < SI_N) {
            double v = X[gl * SI_N + k];
            if (k > 0) {
                double d = 0;
                for (int j = 0; j < k; ++j) d = d + X[gl * SI_N + j] * X[k * SI_N + j];
                v = v - d;
            }
            X[gl * SI_N + k] = v / x;
        }
        __syncthreads();
    }
    if (dst)
        for (int e = gl; e < SI_N * SI_N; e += 16) {
            const int i = e / SI_N, j = e - i * SI_N;
            dst[e] = j >= i ? X[j * SI_N + i] : 0.0;
        }
}

}  // namespace gvx
