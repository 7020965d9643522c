/*
 * fmat.c -- CPU restatement of cv::findFundamentalMat(p1, p2, FM_RANSAC, thresh,
 * 0.99, mask) as Tracking::trackReferenceFrame calls it (tracking/tracking.cc:547-548:
 * undistorted pixel points, thresh = reprojection_error_std_ = 1.5, only when there
 * are >= 15 points).  TEST INFRASTRUCTURE ONLY (see gvx_oracle.h).
 *
 * OpenCV 4.x semantics, recalled from modules/calib3d/src/fundam.cpp, ptsetreg.cpp
 * and modules/core/src/lapack.cpp, mathfuncs.cpp (OpenCV is not vendored; SURVEY
 * 8c) -- parity against OpenCV itself is UNPINNED:
 *   findFundamentalMat   npoints >= 15 and FM_RANSAC -> RANSACPointSetRegistrator
 *                        (modelPoints 7, maxIters 1000), no refinement afterwards
 *   RANSAC run           RNG((uint64)-1); getSubset(maxAttempts 10000): 7 distinct
 *                        uniform indices, the whole subset redrawn while
 *                        FMEstimatorCallback::checkSubset (haveCollinearPoints of the
 *                        last point, both images) fails; findInliers with
 *                        err <= (float)(thresh^2); a model replaces the best when its
 *                        count > max(best, 6), then niters = RANSACUpdateNumIters
 *   run7Point            Hartley normalisation (centroid, mean distance sqrt(2)),
 *                        SVDecomp(A 7x9, MODIFY_A + FULL_UV) = JacobiSVDImpl_ on the
 *                        transposed problem with the null space (rows 7, 8 of Vt)
 *                        completed from RNG(0x12345678) random vectors (two
 *                        Gram-Schmidt passes), the det cubic, solveCubic, F per root
 *                        normalised to F(3,3) = 1, de-normalised T2^T F T1, then
 *                        rescaled by 1 / F(3,3)
 *   computeError         max of the two squared point-to-epipolar-line distances
 *                        (float)
 * Pinned by known answers in tests/test_oracle_fmat.py: exact epipolar geometry of
 * synthetic two-view scenes, the rank-2 / epipolar constraints of every 7-point
 * model, solveCubic against numpy.roots, the MWC generator's recurrence.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "gvx_oracle.h"

#define CV_PI_ 3.1415926535897932384626433832795

/* cv::RNG: multiply-with-carry, CV_RNG_COEFF 4164903690 (core.hpp) */
typedef struct {
    uint64_t state;
} cvrng;
static unsigned rng_next(cvrng* r) {
    r->state = (uint64_t)(unsigned)r->state * 4164903690U + (unsigned)(r->state >> 32);
    return (unsigned)r->state;
}
static int rng_uniform(cvrng* r, int a, int b) { return a == b ? a : (int)(rng_next(r) % (unsigned)(b - a) + a); }

unsigned orc_cvrng_next(uint64_t* state) {
    cvrng r = {*state};
    const unsigned v = rng_next(&r);
    *state = r.state;
    return v;
}

/* haveCollinearPoints (fundam.cpp): the last of `count` points against every pair */
static int have_collinear(const float* p, int count) {
    const int i = count - 1;
    for (int j = 0; j < i; j++) {
        /* Point2f differences: float subtraction, then widened */
        const double dx1 = (double)(p[2 * j] - p[2 * i]), dy1 = (double)(p[2 * j + 1] - p[2 * i + 1]);
        for (int k = 0; k < j; k++) {
            const double dx2 = (double)(p[2 * k] - p[2 * i]), dy2 = (double)(p[2 * k + 1] - p[2 * i + 1]);
            if (fabs(dx2 * dy1 - dy2 * dx1) <= FLT_EPSILON * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2)))
                return 1;
        }
    }
    return 0;
}

/* JacobiSVDImpl_<double> (lapack.cpp) for At: n rows of length m (row stride m),
   n1 output rows (rows n..n1-1 are completed with RNG(0x12345678) vectors), the
   Vt rotations skipped (only U = At is used here: the null space of A 7x9 is in
   rows 7, 8 of the transposed problem's U).  minval DBL_MIN, eps 10 * DBL_EPSILON. */
static void jacobi_svd(double* At, double* W, int m, int n, int n1) {
    const double minval = DBL_MIN, eps = DBL_EPSILON * 10;
    const int max_iter = m > 30 ? m : 30;
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) sd += At[i * m + k] * At[i * m + k];
        W[i] = sd;
    }
    for (int iter = 0; iter < max_iter; iter++) {
        int changed = 0;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                double *Ai = At + i * m, *Aj = At + j * m;
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < m; k++) p += Ai[k] * Aj[k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                const double beta = a - b, gamma = hypot(p, beta);
                double c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                for (int k = 0; k < m; k++) {
                    const double t0 = c * Ai[k] + s * Aj[k];
                    const double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = 1;
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) sd += At[i * m + k] * At[i * m + k];
        W[i] = sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i];
            W[i] = W[j];
            W[j] = t;
            for (int k = 0; k < m; k++) {
                t = At[i * m + k];
                At[i * m + k] = At[j * m + k];
                At[j * m + k] = t;
            }
        }
    }
    cvrng rng = {0x12345678};
    for (int i = 0; i < n1; i++) {
        double sd = i < n ? W[i] : 0;
        for (int ii = 0; ii < 100 && sd <= minval; ii++) {
            const double val0 = 1. / m;
            for (int k = 0; k < m; k++) At[i * m + k] = (rng_next(&rng) & 256) != 0 ? val0 : -val0;
            for (int it = 0; it < 2; it++)
                for (int j = 0; j < i; j++) {
                    sd = 0;
                    for (int k = 0; k < m; k++) sd += At[i * m + k] * At[j * m + k];
                    double asum = 0;
                    for (int k = 0; k < m; k++) {
                        const double t = At[i * m + k] - sd * At[j * m + k];
                        At[i * m + k] = t;
                        asum += fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (int k = 0; k < m; k++) At[i * m + k] *= asum;
                }
            sd = 0;
            for (int k = 0; k < m; k++) sd += At[i * m + k] * At[i * m + k];
            sd = sqrt(sd);
        }
        const double s = sd > minval ? 1 / sd : 0.;
        for (int k = 0; k < m; k++) At[i * m + k] *= s;
    }
}

/* cv::solveCubic (mathfuncs.cpp), double coefficients a0 x^3 + a1 x^2 + a2 x + a3 */
int orc_solve_cubic(const double* coeffs, double* roots) {
    int n = 0;
    double a0 = coeffs[0], a1 = coeffs[1], a2 = coeffs[2], a3 = coeffs[3];
    double x0 = 0., x1 = 0., x2 = 0.;
    if (a0 == 0) {
        if (a1 == 0) {
            if (a2 == 0)
                n = a3 == 0 ? -1 : 0;
            else {
                x0 = -a3 / a2;
                n = 1;
            }
        } else {
            double d = a2 * a2 - 4 * a1 * a3;
            if (d >= 0) {
                d = sqrt(d);
                const double q1 = (-a2 + d) * 0.5;
                const double q2 = (a2 + d) * -0.5;
                if (fabs(q1) > fabs(q2)) {
                    x0 = q1 / a1;
                    x1 = a3 / q1;
                } else {
                    x0 = q2 / a1;
                    x1 = a3 / q2;
                }
                n = d > 0 ? 2 : 1;
            }
        }
    } else {
        a0 = 1. / a0;
        a1 *= a0;
        a2 *= a0;
        a3 *= a0;
        const double Q = (a1 * a1 - 3 * a2) * (1. / 9);
        const double R = (a1 * (2 * a1 * a1 - 9 * a2) + 27 * a3) * (1. / 54);
        const double Qcubed = Q * Q * Q;
        double d = (a1 * a1 * (a2 * a2 - 4 * a1 * a3) + 2 * a2 * (9 * a1 * a3 - 2 * a2 * a2) - 27 * a3 * a3) *
                   (1. / 108);
        if (d > 0) {
            const double theta = acos(R / sqrt(Qcubed));
            const double sqrtQ = sqrt(Q);
            const double t0 = -2 * sqrtQ;
            const double t1 = theta * (1. / 3);
            const double t2 = a1 * (1. / 3);
            x0 = t0 * cos(t1) - t2;
            x1 = t0 * cos(t1 + (2. * CV_PI_ / 3)) - t2;
            x2 = t0 * cos(t1 + (4. * CV_PI_ / 3)) - t2;
            n = 3;
        } else if (d == 0) {
            if (R >= 0) {
                x0 = -2 * pow(R, 1. / 3) - a1 / 3;
                x1 = pow(R, 1. / 3) - a1 / 3;
            } else {
                x0 = 2 * pow(-R, 1. / 3) - a1 / 3;
                x1 = -pow(-R, 1. / 3) - a1 / 3;
            }
            x2 = 0;
            n = x0 == x1 ? 1 : 2;
            x1 = x0 == x1 ? 0 : x1;
        } else {
            d = sqrt(-d);
            double e = pow(d + fabs(R), 1. / 3);
            if (R > 0) e = -e;
            x0 = (e + Q / e) - a1 * (1. / 3);
            n = 1;
        }
    }
    roots[0] = x0;
    roots[1] = x1;
    roots[2] = x2;
    return n;
}

/* 3x3 product C = A B (row-major), sums in k order (cv::gemm for a 3x3) */
static void mul33(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}

/* run7Point (fundam.cpp): m1, m2 = 7 float points each; F = up to 3 row-major 3x3 */
int orc_run7point(const float* m1, const float* m2, double* fmatrix) {
    double a[9 * 9], w[9], c[4], r[3] = {0, 0, 0};
    double m1cx = 0, m1cy = 0, m2cx = 0, m2cy = 0, scale1 = 0, scale2 = 0;
    const int count = 7;
    for (int i = 0; i < count; i++) {
        m1cx += (double)m1[2 * i];
        m1cy += (double)m1[2 * i + 1];
        m2cx += (double)m2[2 * i];
        m2cy += (double)m2[2 * i + 1];
    }
    const double t = 1. / count;
    m1cx *= t;
    m1cy *= t;
    m2cx *= t;
    m2cy *= t;
    for (int i = 0; i < count; i++) {
        const double dx1 = m1[2 * i] - m1cx, dy1 = m1[2 * i + 1] - m1cy;
        const double dx2 = m2[2 * i] - m2cx, dy2 = m2[2 * i + 1] - m2cy;
        scale1 += sqrt(dx1 * dx1 + dy1 * dy1);
        scale2 += sqrt(dx2 * dx2 + dy2 * dy2);
    }
    scale1 *= t;
    scale2 *= t;
    if (scale1 < FLT_EPSILON || scale2 < FLT_EPSILON) return 0;
    scale1 = sqrt(2.) / scale1;
    scale2 = sqrt(2.) / scale2;
    /* rows 0..6 of At = A's rows (the transposed problem: m = 9, n = 7, n1 = 9) */
    memset(a, 0, sizeof a);
    for (int i = 0; i < 7; i++) {
        const double x0 = (m1[2 * i] - m1cx) * scale1;
        const double y0 = (m1[2 * i + 1] - m1cy) * scale1;
        const double x1 = (m2[2 * i] - m2cx) * scale2;
        const double y1 = (m2[2 * i + 1] - m2cy) * scale2;
        double* ai = a + i * 9;
        ai[0] = x1 * x0;
        ai[1] = x1 * y0;
        ai[2] = x1;
        ai[3] = y1 * x0;
        ai[4] = y1 * y0;
        ai[5] = y1;
        ai[6] = x0;
        ai[7] = y0;
        ai[8] = 1;
    }
    jacobi_svd(a, w, 9, 7, 9);
    double* f1 = a + 7 * 9;
    double* f2 = a + 8 * 9;
    for (int i = 0; i < 9; i++) f1[i] -= f2[i];
    double t0 = f2[4] * f2[8] - f2[5] * f2[7];
    double t1 = f2[3] * f2[8] - f2[5] * f2[6];
    double t2 = f2[3] * f2[7] - f2[4] * f2[6];
    c[3] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2;
    c[2] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2 - f1[3] * (f2[1] * f2[8] - f2[2] * f2[7]) +
           f1[4] * (f2[0] * f2[8] - f2[2] * f2[6]) - f1[5] * (f2[0] * f2[7] - f2[1] * f2[6]) +
           f1[6] * (f2[1] * f2[5] - f2[2] * f2[4]) - f1[7] * (f2[0] * f2[5] - f2[2] * f2[3]) +
           f1[8] * (f2[0] * f2[4] - f2[1] * f2[3]);
    t0 = f1[4] * f1[8] - f1[5] * f1[7];
    t1 = f1[3] * f1[8] - f1[5] * f1[6];
    t2 = f1[3] * f1[7] - f1[4] * f1[6];
    c[1] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2 - f2[3] * (f1[1] * f1[8] - f1[2] * f1[7]) +
           f2[4] * (f1[0] * f1[8] - f1[2] * f1[6]) - f2[5] * (f1[0] * f1[7] - f1[1] * f1[6]) +
           f2[6] * (f1[1] * f1[5] - f1[2] * f1[4]) - f2[7] * (f1[0] * f1[5] - f1[2] * f1[3]) +
           f2[8] * (f1[0] * f1[4] - f1[1] * f1[3]);
    c[0] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2;
    const int n = orc_solve_cubic(c, r);
    if (n < 1 || n > 3) return n;
    const double T1[9] = {scale1, 0, -scale1 * m1cx, 0, scale1, -scale1 * m1cy, 0, 0, 1};
    const double T2t[9] = {scale2, 0, 0, 0, scale2, 0, -scale2 * m2cx, -scale2 * m2cy, 1};
    for (int k = 0; k < n; k++, fmatrix += 9) {
        double lambda = r[k], mu = 1.;
        const double s = f1[8] * r[k] + f2[8];
        if (fabs(s) > DBL_EPSILON) {
            mu = 1. / s;
            lambda *= mu;
            fmatrix[8] = 1.;
        } else
            fmatrix[8] = 0.;
        for (int i = 0; i < 8; i++) fmatrix[i] = f1[i] * lambda + f2[i] * mu;
        double tmp[9], F[9];
        mul33(T2t, fmatrix, tmp);
        mul33(tmp, T1, F);
        if (fabs(F[8]) > FLT_EPSILON) {
            const double sc = 1. / F[8];
            for (int i = 0; i < 9; i++) F[i] *= sc;
        }
        memcpy(fmatrix, F, sizeof F);
    }
    return n;
}

/* FMEstimatorCallback::computeError (fundam.cpp) */
void orc_fm_error(int n, const float* m1, const float* m2, const double* F, float* err) {
    for (int i = 0; i < n; i++) {
        const double x1 = m1[2 * i], y1 = m1[2 * i + 1], x2 = m2[2 * i], y2 = m2[2 * i + 1];
        double a = F[0] * x1 + F[1] * y1 + F[2];
        double b = F[3] * x1 + F[4] * y1 + F[5];
        double c = F[6] * x1 + F[7] * y1 + F[8];
        const double s2 = 1. / (a * a + b * b);
        const double d2 = x2 * a + y2 * b + c;
        a = F[0] * x2 + F[3] * y2 + F[6];
        b = F[1] * x2 + F[4] * y2 + F[7];
        c = F[2] * x2 + F[5] * y2 + F[8];
        const double s1 = 1. / (a * a + b * b);
        const double d1 = x1 * a + y1 * b + c;
        const double e1 = d1 * d1 * s1, e2 = d2 * d2 * s2;
        err[i] = (float)(e1 > e2 ? e1 : e2);
    }
}

/* RANSACUpdateNumIters (ptsetreg.cpp) */
int orc_ransac_update_num_iters(double p, double ep, int model_points, int max_iters) {
    p = p > 0. ? p : 0.;
    p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.;
    ep = ep < 1. ? ep : 1.;
    double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
    double denom = 1. - pow(1. - ep, model_points);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)lrint(num / denom);
}

int orc_find_fundamental_ransac(int count, const float* m1, const float* m2, double thresh, double confidence,
                                int max_iters, unsigned char* mask, double* Fout, int* iters_out) {
    if (count < 15) return -1;
    if (thresh <= 0) thresh = 3;
    if (confidence < DBL_EPSILON || confidence > 1 - DBL_EPSILON) confidence = 0.99;
    const int model_points = 7;
    int niters = max_iters > 1 ? max_iters : 1, max_good = 0, iter;
    cvrng rng = {(uint64_t)-1};
    const float t = (float)(thresh * thresh);
    double best_F[9] = {0};
    int best_iter = -1;
    float err[4096];
    float ms1[14], ms2[14];
    if (count > 4096) return -2;
    for (iter = 0; iter < niters; iter++) {
        /* getSubset(m1, m2, ms1, ms2, rng, 10000) */
        int found = 0;
        for (int attempts = 0; attempts < 10000; ++attempts) {
            int idx[7];
            for (int i = 0; i < model_points; ++i) {
                int idx_i, dup;
                do {
                    idx_i = rng_uniform(&rng, 0, count);
                    dup = 0;
                    for (int j = 0; j < i; j++)
                        if (idx[j] == idx_i) dup = 1;
                } while (dup);
                idx[i] = idx_i;
                ms1[2 * i] = m1[2 * idx_i];
                ms1[2 * i + 1] = m1[2 * idx_i + 1];
                ms2[2 * i] = m2[2 * idx_i];
                ms2[2 * i + 1] = m2[2 * idx_i + 1];
            }
            if (have_collinear(ms1, model_points) || have_collinear(ms2, model_points)) continue;
            found = 1;
            break;
        }
        if (!found) {
            if (iter == 0) return 0;
            break;
        }
        double F[27];
        const int nmodels = orc_run7point(ms1, ms2, F);
        if (nmodels <= 0) continue;
        for (int i = 0; i < nmodels; i++) {
            orc_fm_error(count, m1, m2, F + 9 * i, err);
            int good = 0;
            for (int k = 0; k < count; k++) good += err[k] <= t;
            if (good > (max_good > model_points - 1 ? max_good : model_points - 1)) {
                memcpy(best_F, F + 9 * i, sizeof best_F);
                max_good = good;
                best_iter = iter;
                niters = orc_ransac_update_num_iters(confidence, (double)(count - good) / count, model_points, niters);
            }
        }
    }
    if (iters_out) *iters_out = iter;
    (void)best_iter;
    if (max_good <= 0) {
        memset(mask, 0, (size_t)count);
        return 0;
    }
    orc_fm_error(count, m1, m2, best_F, err);
    for (int k = 0; k < count; k++) mask[k] = err[k] <= t;
    if (Fout) memcpy(Fout, best_F, sizeof best_F);
    return 1;
}
