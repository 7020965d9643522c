/*
 * marg.c -- CPU restatement of MarginalizationInfo::marginalization() after the
 * factors are evaluated (TEST INFRASTRUCTURE ONLY; see gvx_oracle.h).  Paths are
 * relative to /root/reference/ic_gvins/ic_gvins/.
 *
 *   orc_marg_construct   constructEquation   factors/marginalization_info.h:195-230
 *                        (with ResidualBlockInfo::Evaluate's loss correction,
 *                        factors/residual_block_info.h:59-87, for a HuberLoss)
 *   orc_marg_schur       schurElimination    factors/marginalization_info.h:170-192
 *   orc_marg_linearize   linearization       factors/marginalization_info.h:153-167
 *   orc_sym_eigen        Eigen::SelfAdjointEigenSolver<MatrixXd>(A) with eigenvectors
 *                        (Eigen >= 3.3.7, README.md:48): scaling to [-1, 1],
 *                        Householder tridiagonalization (tridiagonalization_inplace),
 *                        the Householder sequence evaluated in place into Q, the
 *                        implicit symmetric QR with Wilkinson shift
 *                        (computeFromTridiagonal_impl / tridiagonal_qr_step,
 *                        maxIterations 30) and the selection sort into ascending
 *                        order.  Only the lower triangle of A is read, as in Eigen.
 *
 * Order: each Eigen expression is evaluated in its own order of operations (products
 * formed before they are added, Givens rotations and Householder reflections in
 * Eigen's formulas).  Dense reductions, which Eigen's SIMD kernels reassociate in
 * their own way, use fixed orders here that the device kernels reproduce: the
 * solver's vector sums (squaredNorm, dot, the Householder column dots) are sum64
 * (64 lane-strided partial sums folded by an xor butterfly), its symmetric
 * mat-vec is eig_groups() column chunks folded in order, and every other sum
 * (GEMV / GEMM inner sums, J^T J) is sequential.  So the device results are
 * bit-identical to this restatement, while the restatement sits within
 * reassociation distance (a fp64 tolerance) of Eigen.
 * Parity unpinned against the reference binaries (Eigen and Ceres absent);
 * pinned by numpy (LAPACK) eigen-decompositions, dense normal equations and the
 * Schur-complement identities in tests/test_oracle_marg.py.
 */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "gvx_oracle.h"

#define MARG_EPS 1e-8 /* MarginalizationInfo::EPS (marginalization_info.h:308) */

/* numext::hypot (Eigen/src/Core/MathFunctionsImpl.h positive_real_hypot) */
static double e_hypot(double x, double y) {
    const double ax = fabs(x), ay = fabs(y);
    double p, qp;
    if (ax > ay) {
        p = ax;
        qp = ay / p;
    } else {
        p = ay;
        qp = ax / p;
    }
    if (p == 0.0) return 0.0;
    return p * sqrt(1.0 + qp * qp);
}

/* JacobiRotation<double>::makeGivens(p, q) (Eigen/src/Jacobi/Jacobi.h), real case */
static void make_givens(double p, double q, double* c, double* s) {
    if (q == 0.0) {
        *c = p < 0.0 ? -1.0 : 1.0;
        *s = 0.0;
    } else if (p == 0.0) {
        *c = 0.0;
        *s = q < 0.0 ? 1.0 : -1.0;
    } else if (fabs(p) > fabs(q)) {
        const double t = q / p;
        double u = sqrt(1.0 + t * t);
        if (p < 0.0) u = -u;
        *c = 1.0 / u;
        *s = -t * *c;
    } else {
        const double t = p / q;
        double u = sqrt(1.0 + t * t);
        if (q < 0.0) u = -u;
        *s = -1.0 / u;
        *c = -t * *s;
    }
}

/* Sum of x[0..N): lane-strided partials P_l = sum of x[l], x[l+64], ... in order,
   then P_l <- P_l + P_(l xor o) for o = 32, 16, ..., 1; the result is P_0 (the
   device's per-wave reduction, marg.hip bfly_sum). */
static double sum64(const double* x, int N) {
    double P[64], Q[64];
    for (int l = 0; l < 64; l++) P[l] = 0.0;
    for (int i = 0; i < N; i++) P[i & 63] += x[i];
    for (int o = 32; o > 0; o >>= 1) {
        for (int l = 0; l < 64; l++) Q[l] = P[l] + P[l ^ o];
        memcpy(P, Q, sizeof P);
    }
    return P[0];
}

/* column chunks of the symmetric mat-vec (marg.hip eig_groups) */
static int eig_groups(int rem) {
    const int rpad = (rem + 63) & ~63;
    const int g = 1024 / rpad;
    return g > 16 ? 16 : g;
}

/* tridiagonalization_inplace(matA, hCoeffs) (Eigen/src/Eigenvalues/Tridiagonalization.h):
   a is n x n column-major, lower triangle meaningful.  On return the lower part
   holds the essential Householder vectors below the subdiagonal. */
static void tridiagonalize(int n, double* a, double* hc, double* p, double* x) {
    for (int i = 0; i < n - 1; i++) {
        const int rem = n - i - 1;
        double* col = a + (long)i * n;
        /* makeHouseholderInPlace on v = col[i+1 .. n) */
        const double c0 = col[i + 1];
        for (int k = i + 2; k < n; k++) x[k - i - 2] = col[k] * col[k];
        const double tail = sum64(x, rem - 1);
        double tau, beta;
        if (tail <= DBL_MIN) {
            tau = 0.0;
            beta = c0;
            for (int k = i + 2; k < n; k++) col[k] = 0.0;
        } else {
            beta = sqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
            const double d = c0 - beta;
            for (int k = i + 2; k < n; k++) col[k] = col[k] / d;
            tau = (beta - c0) / beta;
        }
        const double h = tau;
        col[i + 1] = 1.0;
        const double* v = col + i + 1;
        double* S = a + (long)(i + 1) * n + (i + 1); /* bottom-right rem x rem, ld n */
        /* p = A_sub.selfadjointView<Lower>() * (h * v), G column chunks folded in order */
        const int G = eig_groups(rem), chunk = (rem + G - 1) / G;
        for (int j = 0; j < rem; j++) {
            double s = 0.0;
            for (int g = 0; g < G; g++) {
                const int k1 = (g + 1) * chunk < rem ? (g + 1) * chunk : rem;
                double acc = 0.0;
                for (int k = g * chunk; k < k1; k++) {
                    const double ajk = j >= k ? S[(long)k * n + j] : S[(long)j * n + k];
                    acc += ajk * (h * v[k]);
                }
                s += acc;
            }
            p[j] = s;
        }
        for (int k = 0; k < rem; k++) x[k] = p[k] * v[k];
        const double dot = sum64(x, rem);
        const double sc = (h * -0.5) * dot;
        for (int k = 0; k < rem; k++) p[k] += sc * v[k];
        /* rankUpdate(v, p, -1) on the lower triangle */
        for (int k = 0; k < rem; k++) {
            const double a1 = -v[k], a2 = -p[k];
            for (int j = k; j < rem; j++) S[(long)k * n + j] += a1 * p[j] + a2 * v[j];
        }
        col[i + 1] = beta;
        hc[i] = h;
    }
}

/* HouseholderSequence(mat, hCoeffs).setLength(n-1).setShift(1) evaluated into mat
   itself (HouseholderSequence::evalTo, in-place branch), with
   applyHouseholderOnTheLeft (Eigen/src/Householder/Householder.h). */
static void householder_q(int n, double* a, const double* hc, double* tmp, double* x) {
    for (int j = 0; j < n; j++) {
        for (int i = 0; i < j; i++) a[(long)j * n + i] = 0.0;
        a[(long)j * n + j] = 1.0;
    }
    for (int k = n - 2; k >= 0; k--) {
        const int cs = n - k - 1;
        const double tau = hc[k];
        const double* ess = a + (long)k * n + k + 2; /* cs - 1 entries */
        double* C = a + (long)(k + 1) * n + (k + 1);
        if (cs == 1) {
            C[0] *= 1.0 - tau;
        } else if (tau != 0.0) {
            for (int c = 0; c < cs; c++) {
                for (int r = 0; r < cs - 1; r++) x[r] = ess[r] * C[(long)c * n + 1 + r];
                tmp[c] = sum64(x, cs - 1) + C[(long)c * n];
            }
            for (int c = 0; c < cs; c++) C[(long)c * n] -= tau * tmp[c];
            for (int c = 0; c < cs; c++)
                for (int r = 0; r < cs - 1; r++) C[(long)c * n + 1 + r] -= (tau * ess[r]) * tmp[c];
        }
        for (int r = k + 1; r < n; r++) a[(long)k * n + r] = 0.0;
    }
}

/* tridiagonal_qr_step (Eigen/src/Eigenvalues/SelfAdjointEigenSolver.h) with
   Q = Q * G applied to columns k, k+1 (applyOnTheRight with j.transpose()). */
static void qr_step(int n, double* diag, double* sub, int start, int end, double* Q) {
    const double td = (diag[end - 1] - diag[end]) * 0.5;
    const double e = sub[end - 1];
    double mu = diag[end];
    if (td == 0.0) {
        mu -= fabs(e);
    } else {
        const double e2 = e * e;
        const double h = e_hypot(td, e);
        if (e2 == 0.0)
            mu -= (e / (td + (td > 0.0 ? 1.0 : -1.0))) * (e / h);
        else
            mu -= e2 / (td + (td > 0.0 ? h : -h));
    }
    double x = diag[start] - mu;
    double z = sub[start];
    for (int k = start; k < end && z != 0.0; k++) {
        double c, s;
        make_givens(x, z, &c, &s);
        const double sdk = s * diag[k] + c * sub[k];
        const double dkp1 = s * sub[k] + c * diag[k + 1];
        diag[k] = c * (c * diag[k] - s * sub[k]) - s * (c * sub[k] - s * diag[k + 1]);
        diag[k + 1] = s * sdk + c * dkp1;
        sub[k] = c * sdk - s * dkp1;
        if (k > start) sub[k - 1] = c * sub[k - 1] - s * z;
        x = sub[k];
        if (k < end - 1) {
            z = -s * sub[k + 1];
            sub[k + 1] = c * sub[k + 1];
        }
        double* qx = Q + (long)k * n;
        double* qy = Q + (long)(k + 1) * n;
        for (int i = 0; i < n; i++) {
            const double xi = qx[i], yi = qy[i];
            qx[i] = c * xi - s * yi;
            qy[i] = s * xi + c * yi;
        }
    }
}

int orc_sym_eigen(int n, const double* A, int lda, double* w, double* V) {
    if (n <= 0) return 0;
    if (n == 1) {
        w[0] = A[0];
        V[0] = 1.0;
        return 0;
    }
    double scale = 0.0;
    for (int j = 0; j < n; j++)
        for (int i = 0; i < n; i++) {
            const double v = i >= j ? A[(long)j * lda + i] : 0.0;
            V[(long)j * n + i] = v;
            if (fabs(v) > scale) scale = fabs(v);
        }
    if (scale == 0.0) scale = 1.0;
    for (int j = 0; j < n; j++)
        for (int i = j; i < n; i++) V[(long)j * n + i] /= scale;
    double* work = (double*)malloc(sizeof(double) * 4 * (size_t)n);
    double *hc = work, *tmp = work + n, *diag = w, *sub = work + 2 * n, *x = work + 3 * n;
    tridiagonalize(n, V, hc, tmp, x);
    for (int i = 0; i < n; i++) diag[i] = V[(long)i * n + i];
    for (int i = 0; i < n - 1; i++) sub[i] = V[(long)i * n + i + 1];
    householder_q(n, V, hc, tmp, x);

    /* computeFromTridiagonal_impl */
    int end = n - 1, start = 0, info = 0;
    long iter = 0;
    const double zero = DBL_MIN, precision_inv = 1.0 / DBL_EPSILON;
    while (end > 0) {
        for (int i = start; i < end; i++) {
            if (fabs(sub[i]) < zero) {
                sub[i] = 0.0;
            } else {
                const double ss = precision_inv * sub[i];
                if (ss * ss <= fabs(diag[i]) + fabs(diag[i + 1])) sub[i] = 0.0;
            }
        }
        while (end > 0 && sub[end - 1] == 0.0) end--;
        if (end <= 0) break;
        iter++;
        if (iter > 30L * n) {
            info = 1;
            break;
        }
        start = end - 1;
        while (start > 0 && sub[start - 1] != 0.0) start--;
        qr_step(n, diag, sub, start, end, V);
    }
    if (info == 0) {
        for (int i = 0; i < n - 1; i++) {
            int k = i;
            for (int j = i + 1; j < n; j++)
                if (diag[j] < diag[k]) k = j;
            if (k != i) {
                const double t = diag[i];
                diag[i] = diag[k];
                diag[k] = t;
                double* ci = V + (long)i * n;
                double* ck = V + (long)k * n;
                for (int r = 0; r < n; r++) {
                    const double u = ci[r];
                    ci[r] = ck[r];
                    ck[r] = u;
                }
            }
        }
    }
    for (int i = 0; i < n; i++) w[i] *= scale;
    free(work);
    return info;
}

/* ceres::HuberLoss(a)::Evaluate, then ResidualBlockInfo::Evaluate's correction.
   Huber's rho'' is 0 (inlier) or negative (outlier), so the corrector always takes
   its first branch: residual_scaling = sqrt(rho'), alpha_sq_norm = 0, and
   J - 0 * r (r^T J) = J, i.e. every Jacobian block is scaled by sqrt(rho'). */
static double huber_sqrt_rho1(double a, const double* e, int nres) {
    double sq = 0.0;
    for (int k = 0; k < nres; k++) sq += e[k] * e[k];
    double rho1;
    if (sq > a * a) {
        const double r = sqrt(sq);
        rho1 = a / r;
        if (rho1 < DBL_MIN) rho1 = DBL_MIN;
    } else {
        rho1 = 1.0;
    }
    return sqrt(rho1);
}

static int local_size(int size) { return size == 7 ? 6 : size; }

void orc_marg_construct(int n_fac, const int* nres, const int* blk_off, const int* blk, const long* fac_off,
                        const double* data, const double* loss, const int* size, const int* index, int L,
                        double* H0, double* b0) {
    memset(H0, 0, sizeof(double) * (size_t)L * L);
    memset(b0, 0, sizeof(double) * (size_t)L);
    for (int f = 0; f < n_fac; f++) {
        const int R = nres[f], nb = blk_off[f + 1] - blk_off[f];
        const int* bl = blk + blk_off[f];
        const double* src = data + fac_off[f];
        long total = R;
        for (int i = 0; i < nb; i++) total += (long)R * size[bl[i]];
        double* buf = (double*)malloc(sizeof(double) * (size_t)total);
        memcpy(buf, src, sizeof(double) * (size_t)total);
        if (loss && loss[f] > 0.0) {
            const double sr = huber_sqrt_rho1(loss[f], buf, R);
            for (long k = R; k < total; k++) buf[k] = sr * buf[k];
            for (int k = 0; k < R; k++) buf[k] *= sr;
        }
        const double* e = buf;
        const double* J[64];
        long o = R;
        for (int i = 0; i < nb && i < 64; i++) {
            J[i] = buf + o;
            o += (long)R * size[bl[i]];
        }
        for (int i = 0; i < nb; i++) {
            const int gi = size[bl[i]], rows = local_size(gi), row0 = index[bl[i]];
            for (int j = i; j < nb; j++) {
                const int gj = size[bl[j]], cols = local_size(gj), col0 = index[bl[j]];
                for (int a = 0; a < rows; a++)
                    for (int b = 0; b < cols; b++) {
                        double acc = 0.0;
                        for (int r = 0; r < R; r++) acc += J[i][(long)r * gi + a] * J[j][(long)r * gj + b];
                        double* h = H0 + (long)(col0 + b) * L + row0 + a;
                        *h += acc;
                        if (i != j) H0[(long)(row0 + a) * L + col0 + b] = *h;
                    }
            }
            for (int a = 0; a < rows; a++) {
                double acc = 0.0;
                for (int r = 0; r < R; r++) acc += J[i][(long)r * gi + a] * e[r];
                b0[row0 + a] -= acc;
            }
        }
        free(buf);
    }
}

int orc_marg_schur(int L, int m, const double* H0, const double* b0, double* Hp, double* bp) {
    const int r = L - m;
    double* Hmm = (double*)calloc((size_t)m * m + 1, sizeof(double));
    double* V = (double*)malloc(sizeof(double) * ((size_t)m * m + 1));
    double* w = (double*)malloc(sizeof(double) * (size_t)(m > 0 ? m : 1));
    double* Hi = (double*)malloc(sizeof(double) * ((size_t)m * m + 1));
    double* T = (double*)malloc(sizeof(double) * (size_t)r * (m > 0 ? m : 1));
    for (int b = 0; b < m; b++)
        for (int a = 0; a < m; a++) Hmm[(long)b * m + a] = 0.5 * (H0[(long)b * L + a] + H0[(long)a * L + b]);
    const int info = orc_sym_eigen(m, Hmm, m, w, V);
    for (int k = 0; k < m; k++) w[k] = w[k] > MARG_EPS ? 1.0 / w[k] : 0.0;
    /* Hmm_inv = V * diag * V^T */
    for (int b = 0; b < m; b++)
        for (int a = 0; a < m; a++) {
            double acc = 0.0;
            for (int k = 0; k < m; k++) acc += (V[(long)k * m + a] * w[k]) * V[(long)k * m + b];
            Hi[(long)b * m + a] = acc;
        }
    /* T = Hrm * Hmm_inv; Hp = Hrr - T * Hmr; bp = brr - T * bmm */
    for (int b = 0; b < m; b++)
        for (int a = 0; a < r; a++) {
            double acc = 0.0;
            for (int k = 0; k < m; k++) acc += H0[(long)k * L + m + a] * Hi[(long)b * m + k];
            T[(long)b * r + a] = acc;
        }
    for (int b = 0; b < r; b++)
        for (int a = 0; a < r; a++) {
            double acc = 0.0;
            for (int k = 0; k < m; k++) acc += T[(long)k * r + a] * H0[(long)(m + b) * L + k];
            Hp[(long)b * r + a] = H0[(long)(m + b) * L + m + a] - acc;
        }
    for (int a = 0; a < r; a++) {
        double acc = 0.0;
        for (int k = 0; k < m; k++) acc += T[(long)k * r + a] * b0[k];
        bp[a] = b0[m + a] - acc;
    }
    free(Hmm);
    free(V);
    free(w);
    free(Hi);
    free(T);
    return info;
}

int orc_marg_linearize(int r, const double* Hp, const double* bp, double* J0, double* e0, double* eval) {
    double* V = (double*)malloc(sizeof(double) * ((size_t)r * r + 1));
    double* w = (double*)malloc(sizeof(double) * (size_t)(r > 0 ? r : 1));
    const int info = orc_sym_eigen(r, Hp, r, w, V);
    for (int i = 0; i < r; i++) {
        const double S = w[i] > MARG_EPS ? w[i] : 0.0;
        const double Si = w[i] > MARG_EPS ? 1.0 / w[i] : 0.0;
        const double ss = sqrt(S), sis = sqrt(Si);
        for (int j = 0; j < r; j++) J0[(long)j * r + i] = ss * V[(long)i * r + j];
        double acc = 0.0;
        for (int j = 0; j < r; j++) acc += (sis * V[(long)i * r + j]) * -bp[j];
        e0[i] = acc;
        if (eval) eval[i] = w[i];
    }
    free(V);
    free(w);
    return info;
}
