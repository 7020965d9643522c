// dense.hip -- fp64 dense Cholesky kernels for gfx950: the fast path of the
// device marginalisation (MarginalizationInfo::schurElimination / linearization,
// /root/reference/ic_gvins/ic_gvins/factors/marginalization_info.h:153-192) and
// the building blocks of a reduced (Schur) system solve.
//
// The reference inverts Hmm and factors Hp through Eigen's SelfAdjointEigenSolver,
// dropping eigenvalues <= EPS = 1e-8.  When the smallest eigenvalue is above EPS
// (checked here by a Cholesky factorisation of A - EPS*I succeeding: it exists
// iff A - EPS*I is positive definite) that is the plain inverse, and
//   Hp = Hrr - X^T X,  bp = brr - X^T y   with X = L^-1 Hmr, y = L^-1 bm, L L^T = Hmm,
//   J0 = Lp^T,  e0 = -Lp^-1 bp            with Lp Lp^T = Hp,
// which has J0^T J0 = Hp and J0^T e0 = -bp like the reference's J0 = S^1/2 V^T,
// e0 = -S^-1/2 V^T bp: the prior ||e0 + J0 dx||^2 it defines is the same
// function (J0 and e0 differ from the reference's by an orthogonal transform, as
// they would with any other eigen-solver, by eigenvector signs at least).  The
// check's outcome stays on the device: the eigen-solver path (marg.hip) runs
// only where it failed, so no host round trip decides the path.
//
// potrf_kernel   one 1024-thread workgroup: right-looking blocked Cholesky of the
//                lower triangle, 32-column panels factored in LDS, the trailing
//                matrix updated in 4 x 4 register tiles from the panel in LDS.
// trsv_kernel    one wave per right-hand side: forward substitution L x = b in
//                axpy form (lane i owns rows i, i + 64, ...; the pivot of step k
//                comes through v_readlane), the solution stored row-major.
// schur_chol_kernel  Hp = Hrr - X^T X and bp = brr - X^T y, one thread per entry.
// lin_chol_kernel    J0 = Lp^T.
#include <hip/hip_runtime.h>

#include "gvx_internal.h"

namespace gvx {

namespace {

constexpr int PT = 1024;  // potrf threads
constexpr int NB = 32;    // panel width
constexpr int PLD = NB + 1;

// L (n x n column-major, ld n) <- Cholesky factor of the lower triangle of
// A - shift*I (A column-major, ld lda); the strict upper triangle of L is zeroed.
// *fail = 1 when a pivot is not positive (A - shift*I not positive definite).
// Skipped (nothing written) when gate != nullptr and *gate != 0.
__global__ void __launch_bounds__(PT) potrf_kernel(int n, const double* __restrict__ A, int lda, double shift,
                                                   double* __restrict__ L, int* __restrict__ fail,
                                                   const int* __restrict__ gate) {
    __shared__ double P[GVX_EIG_MAX_N * PLD];  // panel rows k0 .. n-1, NB columns
    __shared__ int bad;
    if (gate && *gate != 0) return;
    const int tid = threadIdx.x;
    if (tid == 0) bad = 0;
    for (long idx = tid; idx < (long)n * n; idx += PT) {
        const int i = (int)(idx % n), j = (int)(idx / n);
        L[idx] = i >= j ? A[(long)j * lda + i] - (i == j ? shift : 0.0) : 0.0;
    }
    __syncthreads();
    for (int k0 = 0; k0 < n; k0 += NB) {
        const int nb = min(NB, n - k0), rows = n - k0;
        for (int idx = tid; idx < rows * nb; idx += PT) {
            const int i = idx % rows, c = idx / rows;
            P[i * PLD + c] = L[(long)(k0 + c) * n + k0 + i];
        }
        __syncthreads();
        for (int j = 0; j < nb; ++j) {
            const double d = P[j * PLD + j];
            if (!(d > 0.0)) {  // every thread reads the same pivot
                if (tid == 0) bad = 1;
                break;
            }
            const double piv = sqrt(d), inv = 1.0 / piv;
            // scale column j below the pivot, then the rank-1 update of the panel's
            // later columns (reading the unscaled column: (a/piv)(b/piv) = ab/d)
            for (int idx = tid; idx < (rows - j - 1) * (nb - j - 1); idx += PT) {
                const int c = j + 1 + idx / (rows - j - 1), i = j + 1 + idx % (rows - j - 1);
                if (i >= c) P[i * PLD + c] -= (P[i * PLD + j] * inv) * (P[c * PLD + j] * inv);
            }
            __syncthreads();
            for (int i = j + 1 + tid; i < rows; i += PT) P[i * PLD + j] *= inv;
            if (tid == 0) P[j * PLD + j] = piv;
            __syncthreads();
        }
        __syncthreads();
        if (bad) break;
        for (int idx = tid; idx < rows * nb; idx += PT) {
            const int i = idx % rows, c = idx / rows;
            if (i >= c) L[(long)(k0 + c) * n + k0 + i] = P[i * PLD + c];
        }
        // trailing update of the lower triangle, 4 x 4 tiles: T(i, c) -= sum_t P(i, t) P(c, t)
        const int s = rows - nb;
        if (s > 0) {
            const int nt = (s + 3) / 4;
            const int tiles = nt * (nt + 1) / 2;
            for (int t = tid; t < tiles; t += PT) {
                // t -> (ti, tc) with tc <= ti (row-major over the lower tile triangle)
                int ti = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
                while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
                while (ti * (ti + 1) / 2 > t) --ti;
                const int tc = t - ti * (ti + 1) / 2;
                const int i0 = nb + 4 * ti, c0 = nb + 4 * tc;
                double acc[4][4] = {};
                for (int q = 0; q < nb; ++q) {
                    double a[4], b[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        a[u] = i0 + u < rows ? P[(i0 + u) * PLD + q] : 0.0;
                        b[u] = c0 + u < rows ? P[(c0 + u) * PLD + q] : 0.0;
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u)
#pragma unroll
                        for (int v = 0; v < 4; ++v) acc[u][v] += a[u] * b[v];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        const int i = i0 + u, c = c0 + v;
                        if (i < rows && c < rows && i >= c) L[(long)(k0 + c) * n + k0 + i] -= acc[u][v];
                    }
            }
        }
        __syncthreads();
    }
    if (tid == 0 && fail) *fail = bad;
}

// x = L^-1 b for nrhs right-hand sides, one wave each: b column j at B + j*ldb
// (rows 0..n-1); x stored row-major: X[k * ldx + j].  neg: x = -L^-1 b.
// Skipped when gate != nullptr and *gate != 0.
constexpr int TRSV_ROWS = GVX_EIG_MAX_N / 64;
__global__ void __launch_bounds__(64) trsv_kernel(int n, const double* __restrict__ L, int nrhs,
                                                  const double* __restrict__ B, long ldb, double* __restrict__ X,
                                                  int ldx, int neg, const int* __restrict__ gate) {
    if (gate && *gate != 0) return;
    const int j = blockIdx.x, lane = threadIdx.x;
    if (j >= nrhs) return;
    double x[TRSV_ROWS];
#pragma unroll
    for (int s = 0; s < TRSV_ROWS; ++s) {
        const int i = lane + 64 * s;
        x[s] = i < n ? B[(long)j * ldb + i] : 0.0;
    }
#pragma unroll
    for (int s = 0; s < TRSV_ROWS; ++s) {
        if (64 * s >= n) break;
        for (int kk = 0; kk < 64 && 64 * s + kk < n; ++kk) {
            const int k = 64 * s + kk;
            const double* col = L + (long)k * n;
            // x_k = x_k / L_kk on its lane, then broadcast
            const long long bits = __double_as_longlong(x[s] / col[k]);
            const int lo = __builtin_amdgcn_readlane((int)bits, kk), hi = __builtin_amdgcn_readlane((int)(bits >> 32), kk);
            const double xk = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
            if (lane == kk) x[s] = xk;
#pragma unroll
            for (int t = s; t < TRSV_ROWS; ++t) {
                const int i = lane + 64 * t;
                if (i > k && i < n) x[t] -= col[i] * xk;
            }
        }
    }
#pragma unroll
    for (int s = 0; s < TRSV_ROWS; ++s) {
        const int i = lane + 64 * s;
        if (i < n) X[(long)i * ldx + j] = neg ? -x[s] : x[s];
    }
}

// Hp(a, b) = Hrr(a, b) - sum_k X(k, a) X(k, b), bp(a) = brr(a) - sum_k X(k, a) X(k, r)
// (X row-major m x (r + 1), the last column y = L^-1 bm).  Skipped when *gate != 0.
__global__ void __launch_bounds__(256) schur_chol_kernel(int L, int m, const double* __restrict__ H0,
                                                         const double* __restrict__ b0, const double* __restrict__ X,
                                                         double* __restrict__ Hp, double* __restrict__ bp,
                                                         const int* __restrict__ gate) {
    if (*gate != 0) return;
    const int r = L - m, w = r + 1;
    const int a = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
    if (a >= r) return;
    double acc = 0.0;
    for (int k = 0; k < m; ++k) acc += X[(long)k * w + a] * X[(long)k * w + b];
    if (b < r)
        Hp[(long)b * r + a] = H0[(long)(m + b) * L + m + a] - acc;
    else
        bp[a] = b0[m + a] - acc;
}

// J0 = Lp^T (column-major r x r: J0(i, j) = Lp(j, i)); eval: NaN (not formed).
// Skipped when *gate != 0.
__global__ void __launch_bounds__(256) lin_chol_kernel(int r, const double* __restrict__ Lp, double* __restrict__ J0,
                                                       double* __restrict__ eval, const int* __restrict__ gate) {
    if (*gate != 0) return;
    const int i = blockIdx.x * 256 + threadIdx.x, j = blockIdx.y;
    if (i >= r) return;
    J0[(long)j * r + i] = Lp[(long)i * r + j];
    if (j == 0 && eval) eval[i] = __builtin_nan("");
}

}  // namespace

hipError_t launch_potrf(gvx_ctx* c, int n, const double* A, int lda, double shift, double* L, int* fail,
                        const int* gate) {
    if (n <= 0) return hipSuccess;
    if (n > GVX_EIG_MAX_N) return hipErrorInvalidValue;
    potrf_kernel<<<1, PT, 0, c->stream>>>(n, A, lda, shift, L, fail, gate);
    return hipGetLastError();
}

hipError_t launch_trsv(gvx_ctx* c, int n, const double* L, int nrhs, const double* B, long ldb, double* X, int ldx,
                       bool neg, const int* gate) {
    if (n <= 0 || nrhs <= 0) return hipSuccess;
    if (n > GVX_EIG_MAX_N) return hipErrorInvalidValue;
    trsv_kernel<<<nrhs, 64, 0, c->stream>>>(n, L, nrhs, B, ldb, X, ldx, neg ? 1 : 0, gate);
    return hipGetLastError();
}

hipError_t launch_schur_chol(gvx_ctx* c, int L, int m, const double* H0, const double* b0, const double* X,
                             double* Hp, double* bp, const int* gate) {
    const int r = L - m;
    if (r <= 0) return hipSuccess;
    schur_chol_kernel<<<dim3((r + 255) / 256, r + 1), 256, 0, c->stream>>>(L, m, H0, b0, X, Hp, bp, gate);
    return hipGetLastError();
}

hipError_t launch_lin_chol(gvx_ctx* c, int r, const double* Lp, double* J0, double* eval, const int* gate) {
    if (r <= 0) return hipSuccess;
    lin_chol_kernel<<<dim3((r + 255) / 256, r), 256, 0, c->stream>>>(r, Lp, J0, eval, gate);
    return hipGetLastError();
}

}  // namespace gvx

// ------------------------------------------------ LM step (DENSE_SCHUR)
namespace gvx {
namespace {

// H(i, i) += D_i^2 (H column-major, ld L)
__global__ void __launch_bounds__(256) add_diag_kernel(int L, double* __restrict__ H, const double* __restrict__ D) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < L) H[(long)i * L + i] += D[i] * D[i];
}

// x = L^-T b (one wave, back substitution over the rows of L, column-major ld n)
__global__ void __launch_bounds__(64) trsv_t_kernel(int n, const double* __restrict__ L, const double* __restrict__ b,
                                                    double* __restrict__ x_out, const int* __restrict__ gate) {
    if (gate && *gate != 0) return;
    const int lane = threadIdx.x;
    double x[TRSV_ROWS];
#pragma unroll
    for (int s = 0; s < TRSV_ROWS; ++s) {
        const int i = lane + 64 * s;
        x[s] = i < n ? b[i] : 0.0;
    }
#pragma unroll
    for (int s = TRSV_ROWS - 1; s >= 0; --s) {
        if (64 * s >= n) continue;
        for (int kk = min(63, n - 1 - 64 * s); kk >= 0; --kk) {
            const int k = 64 * s + kk;
            // x_k = x_k / L_kk, then x_i -= L(k, i) x_k for i < k (row k of L)
            const long long bits = __double_as_longlong(x[s] / L[(long)k * n + k]);
            const int lo = __builtin_amdgcn_readlane((int)bits, kk), hi = __builtin_amdgcn_readlane((int)(bits >> 32), kk);
            const double xk = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
            if (lane == kk) x[s] = xk;
#pragma unroll
            for (int t = 0; t <= s; ++t) {
                const int i = lane + 64 * t;
                if (i < k) x[t] -= L[(long)i * n + k] * xk;
            }
        }
    }
#pragma unroll
    for (int s = 0; s < TRSV_ROWS; ++s) {
        const int i = lane + 64 * s;
        if (i < n) x_out[i] = x[s];
    }
}

// t = be - Hef delta_f  (Hef = H0(0..m, m..L), column-major ld L)
__global__ void __launch_bounds__(256) gemv_kernel(int L, int m, const double* __restrict__ H0,
                                                   const double* __restrict__ b0, const double* __restrict__ df,
                                                   double* __restrict__ t) {
    const int a = blockIdx.x * 256 + threadIdx.x;
    if (a >= m) return;
    double acc = 0.0;
    for (int j = 0; j < L - m; ++j) acc += H0[(long)(m + j) * L + a] * df[j];
    t[a] = b0[a] - acc;
}

}  // namespace

hipError_t launch_lm_step(gvx_ctx* c, const MargLaunch& p, const double* D, double* delta, double* S, double* bs,
                          double* tmp) {
    const int m = p.m, r = p.L - m;
    hipError_t e = launch_h0(c, p);
    if (e != hipSuccess) return e;
    if (D) {
        add_diag_kernel<<<(p.L + 255) / 256, 256, 0, c->stream>>>(p.L, p.H0, D);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    // Hee + D = Lm Lm^T; X = Lm^-1 [Hef | be]; S = Hff - X^T X, bs = bf - X^T y
    if ((e = launch_potrf(c, m, p.H0, p.L, 0.0, p.Lm, p.chol, nullptr)) != hipSuccess) return e;
    if ((e = launch_trsv(c, m, p.Lm, r, p.H0 + (size_t)m * p.L, p.L, p.X, r + 1, false, p.chol)) != hipSuccess)
        return e;
    if ((e = launch_trsv(c, m, p.Lm, 1, p.b0, m, p.X + r, r + 1, false, p.chol)) != hipSuccess) return e;
    if ((e = launch_schur_chol(c, p.L, m, p.H0, p.b0, p.X, S, bs, p.chol)) != hipSuccess) return e;
    // S = Lp Lp^T; delta_f = Lp^-T Lp^-1 bs
    if ((e = launch_potrf(c, r, S, r, 0.0, p.Lp, p.chol + 1, p.chol)) != hipSuccess) return e;
    if ((e = launch_trsv(c, r, p.Lp, 1, bs, r, tmp, 1, false, p.chol + 1)) != hipSuccess) return e;
    trsv_t_kernel<<<1, 64, 0, c->stream>>>(r, p.Lp, tmp, delta + m, p.chol + 1);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // delta_e = Lm^-T Lm^-1 (be - Hef delta_f)
    gemv_kernel<<<(m + 255) / 256, 256, 0, c->stream>>>(p.L, m, p.H0, p.b0, delta + m, tmp);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = launch_trsv(c, m, p.Lm, 1, tmp, m, tmp + m, 1, false, p.chol)) != hipSuccess) return e;
    trsv_t_kernel<<<1, 64, 0, c->stream>>>(m, p.Lm, tmp + m, delta, p.chol);
    return hipGetLastError();
}

}  // namespace gvx
