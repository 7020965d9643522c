// dense.hip -- fp64 dense Cholesky kernels for gfx950: the fast path of the
// device marginalisation (MarginalizationInfo::schurElimination / linearization,
// /root/reference/ic_gvins/ic_gvins/factors/marginalization_info.h:153-192) and
// the LM step's DENSE_SCHUR reduced system (ic_gvins.cc:1170-1180).
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
//                lower triangle.  32-column panels in LDS (column-major, so a
//                thread's rows are consecutive addresses), factored in the
//                unscaled outer-product form a_ic -= a_ij a_cj / a_jj (column j is
//                only read in step j: one barrier per step), scaled at the end;
//                the trailing matrix updated in 4 x 4 register tiles.
// trsv_kernel / trsv_t_kernel  one wave per right-hand side, L x = b / L^T x = b
//                by 64-row blocks: the diagonal block in registers (64 steps of a
//                v_readlane broadcast and one fma), the rows after (before) it
//                updated with independent loads.
// schur_chol_kernel  Hp = Hrr - X^T X, bp = brr - X^T y: 32 x 32 output tiles
//                over 32-deep LDS slabs of X.
// lin_chol_kernel    J0 = Lp^T.
#include <hip/hip_runtime.h>

#include "gvx_internal.h"

namespace gvx {

namespace {

constexpr int PT = 1024;                // potrf threads
constexpr int NB = 32;                  // panel width
constexpr int PR = GVX_EIG_MAX_N + 1;   // panel column stride in LDS (doubles)

__device__ __forceinline__ double bcast(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, lane), hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// L (n x n column-major, ld n) <- Cholesky factor of the lower triangle of
// A - shift*I (A column-major, ld lda); the strict upper triangle of L is zeroed.
// *fail = 1 when a pivot is not positive (A - shift*I not positive definite).
// Skipped (nothing written) when gate != nullptr and *gate != 0.
__global__ void __launch_bounds__(PT) potrf_kernel(int n, const double* __restrict__ A, int lda, double shift,
                                                   double* __restrict__ L, int* __restrict__ fail,
                                                   const int* __restrict__ gate) {
    __shared__ double P[NB * PR];  // panel rows k0 .. n-1 (i = row - k0), NB columns, P[c * PR + i]
    __shared__ int bad;
    if (gate && *gate != 0) return;
    const int tid = threadIdx.x;
    if (tid == 0) bad = 0;
    for (long idx = tid; idx < (long)n * n; idx += PT) {
        const int i = (int)(idx % n), j = (int)(idx / n);
        L[idx] = i >= j ? A[(long)j * lda + i] - (i == j ? shift : 0.0) : 0.0;
    }
    __syncthreads();
    // thread t: column tc (+ 32 k) of the panel, rows ti + 32 k
    const int tc = tid >> 5, ti = tid & 31;
    for (int k0 = 0; k0 < n; k0 += NB) {
        const int nb = min(NB, n - k0), rows = n - k0;
        for (int c = tc; c < nb; c += PT / 32)
            for (int i = c + ti; i < rows; i += 32) P[c * PR + i] = L[(long)(k0 + c) * n + k0 + i];
        __syncthreads();
        for (int j = 0; j < nb; ++j) {
            const double d = P[j * PR + j];
            if (!(d > 0.0)) {  // every thread reads the same pivot
                if (tid == 0) bad = 1;
                break;
            }
            const int c = j + 1 + tc;
            if (c < nb) {
                const double f = P[j * PR + c] / d;
                for (int i = c + ti; i < rows; i += 32) P[c * PR + i] -= P[j * PR + i] * f;
            }
            __syncthreads();
        }
        __syncthreads();
        if (bad) break;  // read after a barrier: uniform
        // scale: l_ij = a_ij / sqrt(a_jj)
        for (int j = tc; j < nb; j += PT / 32) {
            const double s = sqrt(P[j * PR + j]), inv = 1.0 / s;
            for (int i = j + 1 + ti; i < rows; i += 32) P[j * PR + i] *= inv;
            if (ti == 0) P[j * PR + j] = s;
        }
        __syncthreads();
        for (int c = tc; c < nb; c += PT / 32)
            for (int i = c + ti; i < rows; i += 32) L[(long)(k0 + c) * n + k0 + i] = P[c * PR + i];
        // trailing update of the lower triangle, 4 x 4 tiles: T(i, c) -= sum_q P(i, q) P(c, q)
        const int s = rows - nb;
        if (s > 0) {
            const int nt = (s + 3) / 4;
            const int tiles = nt * (nt + 1) / 2;
            for (int t = tid; t < tiles; t += PT) {
                int r4 = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
                while ((r4 + 1) * (r4 + 2) / 2 <= t) ++r4;
                while (r4 * (r4 + 1) / 2 > t) --r4;
                const int c4 = t - r4 * (r4 + 1) / 2;
                const int i0 = nb + 4 * r4, c0 = nb + 4 * c4;
                double acc[4][4] = {};
                for (int q = 0; q < nb; ++q) {
                    double a[4], b[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        a[u] = i0 + u < rows ? P[q * PR + i0 + u] : 0.0;
                        b[u] = c0 + u < rows ? P[q * PR + c0 + u] : 0.0;
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

constexpr int TRSV_ROWS = GVX_EIG_MAX_N / 64;

// x = L^-1 b for nrhs right-hand sides, one wave each: b column j at B + j*ldb
// (rows 0..n-1); x stored row-major: X[k * ldx + j].  neg: x = -L^-1 b.
// Skipped when gate != nullptr and *gate != 0.
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
        const int blk = 64 * s;
        if (blk >= n) break;
        const int nk = min(64, n - blk);
        const int row = blk + lane;
        // the diagonal block's entries of this lane's row, and 1 / L_ii
        double d[64];
#pragma unroll
        for (int kk = 0; kk < 64; ++kk) d[kk] = (kk < nk && row < n) ? L[(long)(blk + kk) * n + row] : 0.0;
        const double inv = row < n ? 1.0 / L[(long)row * n + row] : 0.0;
        double xs = x[s];
#pragma unroll
        for (int kk = 0; kk < 64; ++kk) {
            if (kk < nk) {
                const double xk = bcast(xs * inv, kk);
                if (lane == kk) xs = xk;
                if (lane > kk) xs -= d[kk] * xk;
            }
        }
        x[s] = xs;
        // rows of the later blocks: x_i -= sum_k L(i, k) x_k over this block's k
#pragma unroll
        for (int t = s + 1; t < TRSV_ROWS; ++t) {
            if (64 * t >= n) break;
            const int i = 64 * t + lane;
            double acc = 0.0;
            for (int kk = 0; kk < nk; ++kk) acc += (i < n ? L[(long)(blk + kk) * n + i] : 0.0) * bcast(xs, kk);
            x[t] -= acc;
        }
    }
#pragma unroll
    for (int s = 0; s < TRSV_ROWS; ++s) {
        const int i = lane + 64 * s;
        if (i < n) X[(long)i * ldx + j] = neg ? -x[s] : x[s];
    }
}

// Hp(a, b) = Hrr(a, b) - sum_k X(k, a) X(k, b) for b < r, bp(a) = brr(a) - sum_k
// X(k, a) X(k, r) (X row-major m x (r + 1), its last column y = L^-1 bm): one
// 256-thread workgroup per 32 x 32 output tile, 2 x 2 outputs per thread.
// Skipped when *gate != 0.
constexpr int ST = 32;
__global__ void __launch_bounds__(256) schur_chol_kernel(int L, int m, const double* __restrict__ H0,
                                                         const double* __restrict__ b0, const double* __restrict__ X,
                                                         double* __restrict__ Hp, double* __restrict__ bp,
                                                         const int* __restrict__ gate) {
    __shared__ double Xa[ST][ST + 1], Xb[ST][ST + 1];
    if (*gate != 0) return;
    const int r = L - m, w = r + 1;
    const int a0 = blockIdx.x * ST, b0t = blockIdx.y * ST;
    const int tid = threadIdx.x, ta = (tid & 15) * 2, tb = (tid >> 4) * 2;
    double acc[2][2] = {};
    for (int k0 = 0; k0 < m; k0 += ST) {
        for (int e = tid; e < ST * ST; e += 256) {
            const int kk = e / ST, q = e % ST;
            const int k = k0 + kk;
            Xa[kk][q] = (k < m && a0 + q < r) ? X[(long)k * w + a0 + q] : 0.0;
            Xb[kk][q] = (k < m && b0t + q < w) ? X[(long)k * w + b0t + q] : 0.0;
        }
        __syncthreads();
#pragma unroll 8
        for (int kk = 0; kk < ST; ++kk) {
            const double x0 = Xa[kk][ta], x1 = Xa[kk][ta + 1], y0 = Xb[kk][tb], y1 = Xb[kk][tb + 1];
            acc[0][0] += x0 * y0;
            acc[0][1] += x0 * y1;
            acc[1][0] += x1 * y0;
            acc[1][1] += x1 * y1;
        }
        __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
            const int a = a0 + ta + u, b = b0t + tb + v;
            if (a >= r || b > r) continue;
            if (b < r)
                Hp[(long)b * r + a] = H0[(long)(m + b) * L + m + a] - acc[u][v];
            else
                bp[a] = b0[m + a] - acc[u][v];
        }
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

// H(i, i) += D_i^2 (H column-major, ld L)
__global__ void __launch_bounds__(256) add_diag_kernel(int L, double* __restrict__ H, const double* __restrict__ D) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < L) H[(long)i * L + i] += D[i] * D[i];
}

// x = L^-T b (one wave, back substitution by 64-row blocks from the last: lane
// l holds column blk + l of L, rows blk .. blk + 63 -- its diagonal-block row
// entries, a contiguous run -- then the rows of the earlier blocks)
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
        const int blk = 64 * s;
        if (blk >= n) continue;
        const int nk = min(64, n - blk);
        const int col = blk + lane;
        // d[kk] = L(blk + kk, col): row blk + kk of L, this lane's column
        double d[64];
#pragma unroll
        for (int kk = 0; kk < 64; ++kk) d[kk] = (kk < nk && col < n) ? L[(long)col * n + blk + kk] : 0.0;
        const double inv = col < n ? 1.0 / L[(long)col * n + col] : 0.0;
        double xs = x[s];
#pragma unroll
        for (int kk = 63; kk >= 0; --kk) {
            if (kk >= nk) continue;
            const double xk = bcast(xs * inv, kk);
            if (lane == kk) xs = xk;
            if (lane < kk) xs -= d[kk] * xk;
        }
        x[s] = xs;
        // earlier rows: x_i -= sum_k L(k, i) x_k over this block's k (lane i reads
        // its own contiguous run of column i)
#pragma unroll
        for (int t = 0; t < s; ++t) {
            const int i = 64 * t + lane;
            double acc = 0.0;
            for (int kk = 0; kk < nk; ++kk) acc += L[(long)i * n + blk + kk] * bcast(xs, kk);
            x[t] -= acc;
        }
    }
#pragma unroll
    for (int s = 0; s < TRSV_ROWS; ++s) {
        const int i = lane + 64 * s;
        if (i < n) x_out[i] = x[s];
    }
}

// t = be - Hef delta_f  (Hef = H0(0..m, m..L), column-major ld L): a thread per
// row, four independent partial sums
__global__ void __launch_bounds__(256) gemv_kernel(int L, int m, const double* __restrict__ H0,
                                                   const double* __restrict__ b0, const double* __restrict__ df,
                                                   double* __restrict__ t) {
    const int a = blockIdx.x * 256 + threadIdx.x;
    if (a >= m) return;
    const int r = L - m;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    int j = 0;
    for (; j + 4 <= r; j += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] += H0[(long)(m + j + u) * L + a] * df[j + u];
    }
    for (; j < r; ++j) acc[0] += H0[(long)(m + j) * L + a] * df[j];
    t[a] = b0[a] - ((acc[0] + acc[1]) + (acc[2] + acc[3]));
}

// The LM step's failure epilogue: a non-positive pivot in Hee + D (chol[0]) or
// in S (chol[1]) leaves delta undefined -- the S stage is skipped after a failed
// Hee, and the stages after a failed factorisation read factors that were never
// written.  Every delta entry becomes NaN and chol[1] also records a failed
// Hee + D (S was never formed).  All threads read both flags before thread 0
// may set chol[1]; the answer is the same either way.
__global__ void __launch_bounds__(256) lm_fail_kernel(int L, int* __restrict__ chol, double* __restrict__ delta) {
    const int f0 = chol[0], f1 = chol[1];
    if (!(f0 | f1)) return;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < L) delta[i] = __builtin_nan("");
    if (i == 0 && f0 && !f1) chol[1] = 1;
}

// ---- the LM step with a diagonal Hee (MargLaunch::diag_e): one inverse depth per
// landmark, each reprojection factor touching one, as in the reference's window.
// The Cholesky factor of a diagonal matrix is its square root, and the general
// potrf / trsv kernels reduce to exactly these operations on it (sqrt(a_ii), then
// b_i * (1 / l_ii)), without their one-workgroup m <= 512 limit.
// Ld[i] = sqrt(Hee(i, i) + D_i^2); chol[0] = 1 where a pivot is not positive.
__global__ void __launch_bounds__(256) diag_chol_kernel(int m, int L, const double* __restrict__ H0,
                                                        double* __restrict__ Ld, int* __restrict__ chol) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const double a = H0[(long)i * L + i];
    if (!(a > 0.0)) chol[0] = 1;
    Ld[i] = sqrt(a);
}
// X = Ld^-1 [Hef | be] (row-major m x (r + 1)), as trsv_kernel: x = b * (1 / l).
// Skipped when *gate != 0.
__global__ void __launch_bounds__(256) diag_x_kernel(int m, int L, const double* __restrict__ H0,
                                                     const double* __restrict__ b0, const double* __restrict__ Ld,
                                                     double* __restrict__ X, const int* __restrict__ gate) {
    if (*gate != 0) return;
    const int r = L - m;
    const long idx = (long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long)m * (r + 1)) return;
    const int k = (int)(idx / (r + 1)), j = (int)(idx - (long)k * (r + 1));
    const double inv = 1.0 / Ld[k];
    X[idx] = (j < r ? H0[(long)(m + j) * L + k] : b0[k]) * inv;
}
// delta_e = Ld^-T Ld^-1 t (trsv_kernel then trsv_t_kernel: (t * inv) * inv).
// Skipped when *gate != 0.
__global__ void __launch_bounds__(256) diag_back_kernel(int m, const double* __restrict__ Ld,
                                                        const double* __restrict__ t, double* __restrict__ delta,
                                                        const int* __restrict__ gate) {
    if (*gate != 0) return;
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= m) return;
    const double inv = 1.0 / Ld[k];
    delta[k] = (t[k] * inv) * inv;
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
    schur_chol_kernel<<<dim3((r + ST - 1) / ST, (r + 1 + ST - 1) / ST), 256, 0, c->stream>>>(L, m, H0, b0, X, Hp, bp,
                                                                                              gate);
    return hipGetLastError();
}

hipError_t launch_lin_chol(gvx_ctx* c, int r, const double* Lp, double* J0, double* eval, const int* gate) {
    if (r <= 0) return hipSuccess;
    lin_chol_kernel<<<dim3((r + 255) / 256, r), 256, 0, c->stream>>>(r, Lp, J0, eval, gate);
    return hipGetLastError();
}

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
    if (p.diag_e) {
        diag_chol_kernel<<<(m + 255) / 256, 256, 0, c->stream>>>(m, p.L, p.H0, p.Lm, p.chol);
        const long nx = (long)m * (r + 1);
        diag_x_kernel<<<(unsigned)((nx + 255) / 256), 256, 0, c->stream>>>(m, p.L, p.H0, p.b0, p.Lm, p.X, p.chol);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    } else {
        if ((e = launch_potrf(c, m, p.H0, p.L, 0.0, p.Lm, p.chol, nullptr)) != hipSuccess) return e;
        if ((e = launch_trsv(c, m, p.Lm, r, p.H0 + (size_t)m * p.L, p.L, p.X, r + 1, false, p.chol)) != hipSuccess)
            return e;
        if ((e = launch_trsv(c, m, p.Lm, 1, p.b0, m, p.X + r, r + 1, false, p.chol)) != hipSuccess) return e;
    }
    if ((e = launch_schur_chol(c, p.L, m, p.H0, p.b0, p.X, S, bs, p.chol)) != hipSuccess) return e;
    // S = Lp Lp^T; delta_f = Lp^-T Lp^-1 bs
    if ((e = launch_potrf(c, r, S, r, 0.0, p.Lp, p.chol + 1, p.chol)) != hipSuccess) return e;
    if ((e = launch_trsv(c, r, p.Lp, 1, bs, r, tmp, 1, false, p.chol + 1)) != hipSuccess) return e;
    trsv_t_kernel<<<1, 64, 0, c->stream>>>(r, p.Lp, tmp, delta + m, p.chol + 1);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // delta_e = Lm^-T Lm^-1 (be - Hef delta_f)
    gemv_kernel<<<(m + 255) / 256, 256, 0, c->stream>>>(p.L, m, p.H0, p.b0, delta + m, tmp);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (p.diag_e) {
        diag_back_kernel<<<(m + 255) / 256, 256, 0, c->stream>>>(m, p.Lm, tmp, delta, p.chol);
    } else {
        if ((e = launch_trsv(c, m, p.Lm, 1, tmp, m, tmp + m, 1, false, p.chol)) != hipSuccess) return e;
        trsv_t_kernel<<<1, 64, 0, c->stream>>>(m, p.Lm, tmp + m, delta, p.chol);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    lm_fail_kernel<<<(p.L + 255) / 256, 256, 0, c->stream>>>(p.L, p.chol, delta);
    return hipGetLastError();
}

}  // namespace gvx
