// fmat.hip -- cv::findFundamentalMat(p1, p2, FM_RANSAC, thresh, 0.99, mask) on the
// device for gfx950, as Tracking::trackReferenceFrame uses it to drop outliers
// after the reference-point KLT (tracking/tracking.cc:547-555; paths under
// /root/reference/ic_gvins/ic_gvins/).  The CPU restatement, with the OpenCV 4.x
// sources it follows, is oracle/fmat.c.
//
// One workgroup (4 waves) per point set.  OpenCV's RANSAC is sequential, but the
// subsets it tries are fixed by the RNG stream alone (the results only decide
// when it stops), so the kernel works in batches of 64 hypotheses:
//   1. wave 0 draws the next 64 subsets exactly as getSubset does (MWC RNG,
//      distinct indices, the collinearity check of the 7th point lane-parallel);
//   2. lane h of wave 0 runs run7Point on subset h (Hartley normalisation,
//      OpenCV's one-sided Jacobi SVD with its RNG(0x12345678) null-space
//      completion, the det cubic, 1-3 models) -- the 64 dependent fp64 chains
//      run side by side in the lanes, At in lane-interleaved LDS;
//   3. all 4 waves count the inliers of every (hypothesis, model), a wave per
//      pair, lanes over the points (ballot + popcount);
//   4. lane 0 replays RANSAC's bookkeeping over the batch in order (best model,
//      RANSACUpdateNumIters) and stops where OpenCV's loop would.
// The final mask is recomputed from the best model (the same arithmetic).
#include <hip/hip_runtime.h>

#include <cfloat>

#include "gvx_internal.h"

namespace gvx {

namespace {

constexpr int FM_THREADS = 256;
constexpr int HB = 64;  // hypotheses per batch (the lanes of wave 0)
constexpr double CV_PI_D = 3.1415926535897932384626433832795;

struct FmShared {
    double at[81 * HB];      // At (9 rows x 9) of hypothesis h at [(r*9 + k)*64 + h]
    double F[HB * 27];       // up to 3 row-major models per hypothesis
    double bestF[9];
    int idx[HB * 7];
    int nmodels[HB];
    int cnt[HB * 3];
    int n_valid;             // hypotheses of the batch with a subset
    int fail;                // getSubset failed after n_valid subsets
    int done;
    int max_good;
};

__device__ inline unsigned rng_next(unsigned long long& st) {
    st = (unsigned long long)(unsigned)st * 4164903690ULL + (unsigned)(st >> 32);
    return (unsigned)st;
}

// x % d for the fixed d of a problem: q_est = floor(x * floor(2^32/d) / 2^32)
// undershoots floor(x/d) by at most 1, so one conditional subtraction is exact
__device__ inline unsigned fast_mod(unsigned x, unsigned d, unsigned minv) {
    const unsigned q = __umulhi(x, minv);
    unsigned r = x - q * d;
    if (r >= d) r -= d;
    return r;
}

#define AT(r, k) S.at[((r) * 9 + (k)) * HB + lane]

// run7Point (fundam.cpp) for lane `lane`'s subset; models to S.F[lane*27 ..]
__device__ int run7point(FmShared& S, int lane, const float2* __restrict__ m1p, const float2* __restrict__ m2p) {
    float2 m1[7], m2[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        const int id = S.idx[lane * 7 + i];
        m1[i] = m1p[id];
        m2[i] = m2p[id];
    }
    double m1cx = 0, m1cy = 0, m2cx = 0, m2cy = 0, scale1 = 0, scale2 = 0;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        m1cx += (double)m1[i].x;
        m1cy += (double)m1[i].y;
        m2cx += (double)m2[i].x;
        m2cy += (double)m2[i].y;
    }
    const double t = 1. / 7;
    m1cx *= t;
    m1cy *= t;
    m2cx *= t;
    m2cy *= t;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        const double dx1 = m1[i].x - m1cx, dy1 = m1[i].y - m1cy;
        const double dx2 = m2[i].x - m2cx, dy2 = m2[i].y - m2cy;
        scale1 += sqrt(dx1 * dx1 + dy1 * dy1);
        scale2 += sqrt(dx2 * dx2 + dy2 * dy2);
    }
    scale1 *= t;
    scale2 *= t;
    if (scale1 < FLT_EPSILON || scale2 < FLT_EPSILON) return 0;
    scale1 = sqrt(2.) / scale1;
    scale2 = sqrt(2.) / scale2;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        const double x0 = (m1[i].x - m1cx) * scale1;
        const double y0 = (m1[i].y - m1cy) * scale1;
        const double x1 = (m2[i].x - m2cx) * scale2;
        const double y1 = (m2[i].y - m2cy) * scale2;
        AT(i, 0) = x1 * x0;
        AT(i, 1) = x1 * y0;
        AT(i, 2) = x1;
        AT(i, 3) = y1 * x0;
        AT(i, 4) = y1 * y0;
        AT(i, 5) = y1;
        AT(i, 6) = x0;
        AT(i, 7) = y0;
        AT(i, 8) = 1;
    }
    // ---- JacobiSVDImpl_<double>(At, W, Vt, m = 9, n = 7, n1 = 9, DBL_MIN, 10 DBL_EPSILON)
    constexpr int m = 9, n = 7, n1 = 9;
    const double minval = DBL_MIN, eps = DBL_EPSILON * 10;
    double W[7];
#pragma unroll
    for (int i = 0; i < n; ++i) {
        double sd = 0;
        for (int k = 0; k < m; ++k) sd += AT(i, k) * AT(i, k);
        W[i] = sd;
    }
    for (int iter = 0; iter < 30; ++iter) {
        bool changed = false;
#pragma unroll
        for (int i = 0; i < n - 1; ++i)
#pragma unroll
            for (int j = i + 1; j < n; ++j) {
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < m; ++k) p += AT(i, k) * AT(j, k);
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
                for (int k = 0; k < m; ++k) {
                    const double ai = AT(i, k), aj = AT(j, k);
                    const double t0 = c * ai + s * aj;
                    const double t1 = -s * ai + c * aj;
                    AT(i, k) = t0;
                    AT(j, k) = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = true;
            }
        if (!changed) break;
    }
#pragma unroll
    for (int i = 0; i < n; ++i) {
        double sd = 0;
        for (int k = 0; k < m; ++k) sd += AT(i, k) * AT(i, k);
        W[i] = sqrt(sd);
    }
#pragma unroll
    for (int i = 0; i < n - 1; ++i) {
        int j = i;
        double wj = W[i];
#pragma unroll
        for (int k = i + 1; k < n; ++k)
            if (wj < W[k]) {
                j = k;
                wj = W[k];
            }
        if (i != j) {
            // swap W[i], W[j] and rows i, j (j is lane-varying: select through a loop)
#pragma unroll
            for (int k = i + 1; k < n; ++k)
                if (k == j) {
                    W[k] = W[i];
                    W[i] = wj;
                }
            for (int k = 0; k < m; ++k) {
                const double tt = AT(i, k);
                AT(i, k) = AT(j, k);
                AT(j, k) = tt;
            }
        }
    }
    unsigned long long rs = 0x12345678ULL;
#pragma unroll
    for (int i = 0; i < n1; ++i) {
        double sd = i < n ? W[i] : 0;
        for (int ii = 0; ii < 100 && sd <= minval; ++ii) {
            const double val0 = 1. / m;
            for (int k = 0; k < m; ++k) AT(i, k) = (rng_next(rs) & 256) != 0 ? val0 : -val0;
            for (int it = 0; it < 2; ++it)
                for (int j = 0; j < i; ++j) {
                    sd = 0;
                    for (int k = 0; k < m; ++k) sd += AT(i, k) * AT(j, k);
                    double asum = 0;
                    for (int k = 0; k < m; ++k) {
                        const double tt = AT(i, k) - sd * AT(j, k);
                        AT(i, k) = tt;
                        asum += fabs(tt);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (int k = 0; k < m; ++k) AT(i, k) *= asum;
                }
            sd = 0;
            for (int k = 0; k < m; ++k) sd += AT(i, k) * AT(i, k);
            sd = sqrt(sd);
        }
        const double s = sd > minval ? 1 / sd : 0.;
        for (int k = 0; k < m; ++k) AT(i, k) *= s;
    }
    // ---- the det(lambda f1 + (1 - lambda) f2) = 0 cubic
    double f1[9], f2[9], c[4], r[3] = {0, 0, 0};
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        f2[k] = AT(8, k);
        f1[k] = AT(7, k) - f2[k];
    }
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
    // ---- solveCubic (mathfuncs.cpp)
    int nr = 0;
    {
        double a0 = c[0], a1 = c[1], a2 = c[2], a3 = c[3];
        double x0 = 0., x1 = 0., x2 = 0.;
        if (a0 == 0) {
            if (a1 == 0) {
                if (a2 == 0)
                    nr = a3 == 0 ? -1 : 0;
                else {
                    x0 = -a3 / a2;
                    nr = 1;
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
                    nr = d > 0 ? 2 : 1;
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
                const double u0 = -2 * sqrtQ;
                const double u1 = theta * (1. / 3);
                const double u2 = a1 * (1. / 3);
                x0 = u0 * cos(u1) - u2;
                x1 = u0 * cos(u1 + (2. * CV_PI_D / 3)) - u2;
                x2 = u0 * cos(u1 + (4. * CV_PI_D / 3)) - u2;
                nr = 3;
            } else if (d == 0) {
                if (R >= 0) {
                    x0 = -2 * pow(R, 1. / 3) - a1 / 3;
                    x1 = pow(R, 1. / 3) - a1 / 3;
                } else {
                    x0 = 2 * pow(-R, 1. / 3) - a1 / 3;
                    x1 = -pow(-R, 1. / 3) - a1 / 3;
                }
                x2 = 0;
                nr = x0 == x1 ? 1 : 2;
                x1 = x0 == x1 ? 0 : x1;
            } else {
                d = sqrt(-d);
                double e = pow(d + fabs(R), 1. / 3);
                if (R > 0) e = -e;
                x0 = (e + Q / e) - a1 * (1. / 3);
                nr = 1;
            }
        }
        r[0] = x0;
        r[1] = x1;
        r[2] = x2;
    }
    if (nr < 1 || nr > 3) return nr < 0 ? nr : 0;
    const double T1[9] = {scale1, 0, -scale1 * m1cx, 0, scale1, -scale1 * m1cy, 0, 0, 1};
    const double T2t[9] = {scale2, 0, 0, 0, scale2, 0, -scale2 * m2cx, -scale2 * m2cy, 1};
    double* out = S.F + lane * 27;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (k >= nr) break;
        double lambda = r[k], mu = 1.;
        const double s = f1[8] * r[k] + f2[8];
        double f[9];
        if (fabs(s) > DBL_EPSILON) {
            mu = 1. / s;
            lambda *= mu;
            f[8] = 1.;
        } else {
            f[8] = 0.;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] = f1[i] * lambda + f2[i] * mu;
        double tmp[9], F[9];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                tmp[i * 3 + j] = T2t[i * 3] * f[j] + T2t[i * 3 + 1] * f[3 + j] + T2t[i * 3 + 2] * f[6 + j];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                F[i * 3 + j] = tmp[i * 3] * T1[j] + tmp[i * 3 + 1] * T1[3 + j] + tmp[i * 3 + 2] * T1[6 + j];
        if (fabs(F[8]) > FLT_EPSILON) {
            const double sc = 1. / F[8];
#pragma unroll
            for (int i = 0; i < 9; ++i) F[i] *= sc;
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) out[k * 9 + i] = F[i];
    }
    return nr;
}
#undef AT

// FMEstimatorCallback::computeError for one point
__device__ inline float fm_err(const double* F, float2 p, float2 q) {
    const double x1 = p.x, y1 = p.y, x2 = q.x, y2 = q.y;
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
    return (float)(e1 > e2 ? e1 : e2);
}

// RANSACUpdateNumIters (ptsetreg.cpp)
__device__ int update_num_iters(double p, double ep, int model_points, int max_iters) {
    p = fmax(p, 0.);
    p = fmin(p, 1.);
    ep = fmax(ep, 0.);
    ep = fmin(ep, 1.);
    double num = fmax(1. - p, DBL_MIN);
    double denom = 1. - pow(1. - ep, (double)model_points);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return denom >= 0 || -num >= max_iters * (-denom) ? max_iters : (int)rint(num / denom);
}

__global__ void __launch_bounds__(FM_THREADS)
    fm_ransac_kernel(int n_prob, const int32_t* __restrict__ off, const float2* __restrict__ p1,
                     const float2* __restrict__ p2, float t, double confidence, int max_iters,
                     uint8_t* __restrict__ mask, double* __restrict__ Fout, int32_t* __restrict__ result,
                     unsigned long long* __restrict__ ts) {
    __shared__ FmShared S;
    const int prob = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int o = off[prob], count = off[prob + 1] - o;
    const float2* m1 = p1 + o;
    const float2* m2 = p2 + o;
    uint8_t* mk = mask + o;

    if (count < 15) {  // the reference only calls it with >= 15 points (tracking.cc:547)
        for (int i = tid; i < count; i += FM_THREADS) mk[i] = 1;
        if (tid == 0) result[prob] = -1;
        return;
    }
    const unsigned minv = (unsigned)(0x100000000ULL / (unsigned)count);
    // RANSACPointSetRegistrator::run state (wave 0, uniform)
    unsigned long long rng = ~0ULL;  // RNG((uint64)-1)
    int iter = 0, niters = max_iters > 1 ? max_iters : 1, max_good = 0;
    int batch = 0;
    // ts (nullable, diagnostics): wall clock (100 MHz) per phase of the first 4 batches
#define FM_STAMP(k) \
    if (ts && tid == 0 && prob == 0 && batch < 4) ts[batch * 5 + (k)] = wall_clock64()
    for (;; ++batch) {
        FM_STAMP(0);
        // ---- 1. the next HB subsets (getSubset, maxAttempts 10000)
        if (wid == 0) {
            int nv = 0, fail = 0;
            for (; nv < HB; ++nv) {
                int found = 0;
                for (int attempts = 0; attempts < 10000; ++attempts) {
                    int id[7];
#pragma unroll
                    for (int i = 0; i < 7; ++i) {
                        int v;
                        bool dup;
                        do {
                            v = (int)fast_mod(rng_next(rng), (unsigned)count, minv);
                            dup = false;
#pragma unroll
                            for (int j = 0; j < i; ++j) dup |= id[j] == v;
                        } while (dup);
                        id[i] = v;
                    }
                    // haveCollinearPoints of point 6 against pairs (k < j < 6): 15 pairs per image
                    bool col = false;
                    if (lane < 30) {
                        const int pr = lane % 15;
                        int j = 1, k = pr;
                        while (k >= j) {
                            k -= j;
                            ++j;
                        }
                        const float2* P = lane < 15 ? m1 : m2;
                        const float2 pi = P[id[6]], pj = P[id[j]], pk = P[id[k]];
                        const double dx1 = (double)(pj.x - pi.x), dy1 = (double)(pj.y - pi.y);
                        const double dx2 = (double)(pk.x - pi.x), dy2 = (double)(pk.y - pi.y);
                        col = fabs(dx2 * dy1 - dy2 * dx1) <= FLT_EPSILON * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2));
                    }
                    if (__ballot(col)) continue;
                    if (lane == 0) {
#pragma unroll
                        for (int i = 0; i < 7; ++i) S.idx[nv * 7 + i] = id[i];
                    }
                    found = 1;
                    break;
                }
                if (!found) {
                    fail = 1;
                    break;
                }
            }
            if (lane == 0) {
                S.n_valid = nv;
                S.fail = fail;
            }
        }
        __syncthreads();
        FM_STAMP(1);
        const int nv = S.n_valid;
        // ---- 2. run7Point, one hypothesis per lane of wave 0
        if (wid == 0) {
            int nm = 0;
            if (lane < nv) nm = run7point(S, lane, m1, m2);
            S.nmodels[lane] = nm;
        }
        __syncthreads();
        FM_STAMP(2);
        // ---- 3. inlier counts, a wave per (hypothesis, model), lanes over the points
        for (int q = wid; q < nv * 3; q += FM_THREADS / 64) {
            const int h = q / 3, mdl = q % 3;
            if (mdl >= S.nmodels[h]) continue;
            const double* F = S.F + h * 27 + mdl * 9;
            int good = 0;
            for (int i0 = 0; i0 < count; i0 += 64) {
                const int i = i0 + lane;
                bool in = false;
                if (i < count) in = fm_err(F, m1[i], m2[i]) <= t;
                good += __popcll(__ballot(in));
            }
            if (lane == 0) S.cnt[q] = good;
        }
        __syncthreads();
        FM_STAMP(3);
        // ---- 4. RANSAC's loop over the batch, in order
        if (tid == 0) {
            int h = 0;
            for (; h < nv && iter < niters; ++h, ++iter) {
                for (int mdl = 0; mdl < S.nmodels[h]; ++mdl) {
                    const int good = S.cnt[h * 3 + mdl];
                    if (good > (max_good > 6 ? max_good : 6)) {
#pragma unroll
                        for (int i = 0; i < 9; ++i) S.bestF[i] = S.F[h * 27 + mdl * 9 + i];
                        max_good = good;
                        niters = update_num_iters(confidence, (double)(count - good) / count, 7, niters);
                    }
                }
            }
            // stop: iterations exhausted, or getSubset failed at this iteration
            S.done = iter >= niters || (h == nv && S.fail);
            S.max_good = max_good;
        }
        __syncthreads();
        FM_STAMP(4);
        // S.done is next written in the next batch's step 4, three barriers away
        if (S.done) break;
    }
#undef FM_STAMP
    if (ts && tid == 0 && prob == 0) ts[20] = batch + 1;
    // ---- the mask of the best model
    const int mg = S.max_good;
    if (mg > 0) {
        for (int i = tid; i < count; i += FM_THREADS) mk[i] = fm_err(S.bestF, m1[i], m2[i]) <= t;
        if (tid < 9 && Fout) Fout[(long)prob * 9 + tid] = S.bestF[tid];
    } else {
        for (int i = tid; i < count; i += FM_THREADS) mk[i] = 0;
    }
    if (tid == 0) result[prob] = mg > 0 ? 1 : 0;
}

}  // namespace

hipError_t launch_fm_ransac(gvx_ctx* c, int n_prob, const int32_t* off, const float* p1, const float* p2,
                            double thresh, double confidence, int max_iters, uint8_t* mask, double* F,
                            int32_t* result, unsigned long long* ts) {
    if (n_prob <= 0) return hipSuccess;
    if (thresh <= 0) thresh = 3;
    if (confidence < DBL_EPSILON || confidence > 1 - DBL_EPSILON) confidence = 0.99;
    fm_ransac_kernel<<<n_prob, FM_THREADS, 0, c->stream>>>(n_prob, off, reinterpret_cast<const float2*>(p1),
                                                          reinterpret_cast<const float2*>(p2), (float)(thresh * thresh),
                                                          confidence, max_iters, mask, F, result, ts);
    return hipGetLastError();
}

}  // namespace gvx
