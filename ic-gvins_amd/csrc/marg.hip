// marg.hip -- MarginalizationInfo::marginalization() on the device for gfx950
// (fp64), after the residual blocks are evaluated (the device
// Schur complement).  Paths under /root/reference/ic_gvins/ic_gvins/:
//   constructEquation   factors/marginalization_info.h:195-230  -> h0_kernel
//   schurElimination    factors/marginalization_info.h:170-192  -> sym_eigen_kernel,
//                                                                  hinv_kernel, schur_t_kernel,
//                                                                  schur_p_kernel
//   linearization       factors/marginalization_info.h:153-167  -> sym_eigen_kernel,
//                                                                  linearize_kernel
// The CPU restatement is oracle/marg.c; both follow Eigen's algorithms, and the
// sums that Eigen's SIMD kernels reassociate are plain ordered sums in both, so
// parity is a fp64 tolerance.
//
// h0_kernel: one workgroup per lower block pair (P, Q) of H0 and one per block of
//   b0; a thread owns one entry and walks the pair's contributions in factor
//   order (host-built lists), so H0 = sum_f J_P^T J_Q is formed in the reference's
//   order, each factor's product before it is added, and written to both (P, Q)
//   and (Q, P) -- the exact symmetry constructEquation's transposed copy gives.
// sym_eigen_kernel: Eigen::SelfAdjointEigenSolver<MatrixXd> in ONE workgroup of
//   1024 threads (a latency item: once per keyframe, n = 100-500): scaling to
//   [-1, 1], Householder tridiagonalization (matrix kept symmetric in full storage
//   in global memory / L2 so the symmetric mat-vec and the rank-2 update are
//   coalesced column walks; every sum is one thread's sequential loop, in
//   oracle/marg.c's order, so the two agree bit for bit), Q accumulated in
//   place, then the implicit QR sweeps:
//   wave 0 runs the scalar Givens chain of sweep s+1 while waves 1-15 apply the
//   rotations of sweep s to the rows of Q (a row's rotations need no other row,
//   so a sweep costs one barrier), and finally the selection sort.
// hinv / schur_t / schur_p / linearize: one thread per output entry, ordered
//   inner sums (K <= a few hundred): coalesced over the row index, the other
//   operand broadcast.
#include <hip/hip_runtime.h>

#include <cfloat>

#include "gvx_internal.h"

namespace gvx {

namespace {

constexpr int H0_THREADS = 128;
constexpr int EIG_THREADS = 1024;
constexpr int EIG_WAVES = EIG_THREADS / 64;
constexpr double MARG_EPS = 1e-8;  // MarginalizationInfo::EPS (marginalization_info.h:308)

__device__ inline double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}

// ------------------------------------------------------------- H0 and b0
// c.x = offset of block P's Jacobian (row-major nres x gp) in data, c.y = offset
// of block Q's Jacobian (or of the residuals for a b0 record), c.z = gp | gq << 8 |
// nres << 16, c.w = factor id (loss scale).
__global__ void __launch_bounds__(H0_THREADS) h0_kernel(int n_pairs, const MargPairRec* __restrict__ pairs,
                                                        const int4* __restrict__ contrib,
                                                        const double* __restrict__ data,
                                                        const double* __restrict__ sr, int L,
                                                        double* __restrict__ H0, double* __restrict__ b0) {
    const MargPairRec pr = pairs[blockIdx.x];
    const int n_ent = pr.lp * pr.lq;
    for (int e = threadIdx.x; e < n_ent; e += H0_THREADS) {
        const int a = e % pr.lp, b = e / pr.lp;
        double h = 0.0;
        for (int ci = pr.c0; ci < pr.c1; ++ci) {
            const int4 c = contrib[ci];
            const int gp = c.z & 255, gq = (c.z >> 8) & 255, nres = c.z >> 16;
            const double s = sr ? sr[c.w] : 1.0;
            const double* jp = data + c.x + a;
            const double* jq = data + c.y + (blockIdx.x < n_pairs ? b : 0);
            double acc = 0.0;
            for (int r = 0; r < nres; ++r) acc += (s * jp[(long)r * gp]) * (s * jq[(long)r * gq]);
            if (blockIdx.x < n_pairs)
                h += acc;
            else
                h -= acc;
        }
        if (blockIdx.x < n_pairs) {
            H0[(long)(pr.col0 + b) * L + pr.row0 + a] = h;
            H0[(long)(pr.row0 + a) * L + pr.col0 + b] = h;
        } else {
            b0[pr.row0 + a] = h;
        }
    }
}

// per-factor sqrt(rho') of a HuberLoss (ResidualBlockInfo::Evaluate, residual_block_info.h:59-87)
__global__ void __launch_bounds__(64) loss_kernel(int n_fac, const int32_t* __restrict__ nres,
                                                  const int64_t* __restrict__ res_off,
                                                  const double* __restrict__ loss, const double* __restrict__ data,
                                                  double* __restrict__ sr) {
    const int f = blockIdx.x * 64 + threadIdx.x;
    if (f >= n_fac) return;
    const double a = loss[f];
    if (!(a > 0.0)) {
        sr[f] = 1.0;
        return;
    }
    const double* e = data + res_off[f];
    double sq = 0.0;
    for (int k = 0; k < nres[f]; ++k) sq += e[k] * e[k];
    double rho1 = 1.0;
    if (sq > a * a) rho1 = fmax(DBL_MIN, a / sqrt(sq));
    sr[f] = sqrt(rho1);
}

// ------------------------------------------------------------ eigen solver
struct EigShared {
    double v[GVX_EIG_MAX_N];
    double p[GVX_EIG_MAX_N];
    double part[EIG_THREADS];
    double diag[GVX_EIG_MAX_N];
    double sub[GVX_EIG_MAX_N];
    double rc[2][GVX_EIG_MAX_N];
    double rs[2][GVX_EIG_MAX_N];
    double red[EIG_WAVES];
    double sc[2];
    int sw[2][2];  // per rotation buffer: first column, rotation count (-1: no more sweeps)
    int swap[GVX_EIG_MAX_N];
};

// JacobiRotation<double>::makeGivens (Eigen/src/Jacobi/Jacobi.h), real case
__device__ inline void make_givens(double p, double q, double& c, double& s) {
    if (q == 0.0) {
        c = p < 0.0 ? -1.0 : 1.0;
        s = 0.0;
    } else if (p == 0.0) {
        c = 0.0;
        s = q < 0.0 ? 1.0 : -1.0;
    } else if (fabs(p) > fabs(q)) {
        const double t = q / p;
        double u = sqrt(1.0 + t * t);
        if (p < 0.0) u = -u;
        c = 1.0 / u;
        s = -t * c;
    } else {
        const double t = p / q;
        double u = sqrt(1.0 + t * t);
        if (q < 0.0) u = -u;
        s = -1.0 / u;
        c = -t * s;
    }
}

__device__ inline double e_hypot(double x, double y) {
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

// Producer state of computeFromTridiagonal_impl (wave 0, uniform).
struct QrState {
    int start, end;
    long iter;
    int info;
};

// One turn of computeFromTridiagonal_impl's loop up to and including one
// tridiagonal_qr_step, whose rotations go to buffer b.  Wave 0 only.
__device__ void qr_produce(EigShared& S, QrState& st, int n, int b, int lane) {
    double* D = S.diag;
    double* E = S.sub;
    const double zero = DBL_MIN, precision_inv = 1.0 / DBL_EPSILON;
    for (;;) {
        for (int i = st.start + lane; i < st.end; i += 64) {
            const double ei = E[i];
            if (fabs(ei) < zero) {
                E[i] = 0.0;
            } else {
                const double ss = precision_inv * ei;
                if (ss * ss <= fabs(D[i]) + fabs(D[i + 1])) E[i] = 0.0;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // while (end > 0 && sub[end-1] == 0) end--;  (64 entries per ballot)
        while (st.end > 0) {
            const int i = st.end - 1 - lane;
            const bool nz = i >= 0 && E[i] != 0.0;
            const unsigned long long m = __ballot(nz);
            if (m) {
                st.end -= __builtin_ctzll(m);
                break;
            }
            st.end -= 64;
            if (st.end < 0) st.end = 0;
        }
        if (st.end <= 0) {
            if (lane == 0) S.sw[b][1] = -1;
            return;
        }
        st.iter++;
        if (st.iter > 30L * n) {
            st.info = 1;
            if (lane == 0) S.sw[b][1] = -1;
            return;
        }
        // start = end - 1; while (start > 0 && sub[start-1] != 0) start--;
        st.start = st.end - 1;
        while (st.start > 0) {
            const int i = st.start - 1 - lane;
            const bool z = i < 0 || E[i] == 0.0;
            const unsigned long long m = __ballot(z);
            if (m) {
                st.start -= __builtin_ctzll(m);
                break;
            }
            st.start -= 64;
        }
        // tridiagonal_qr_step(diag, subdiag, start, end)
        const int start = st.start, end = st.end;
        const double td = (D[end - 1] - D[end]) * 0.5;
        const double e = E[end - 1];
        double mu = D[end];
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
        double dk = D[start], ek = E[start];
        double x = dk - mu, z = ek;
        double eprev = 0.0;
        int k = start;
        for (; k < end && z != 0.0; ++k) {
            const double dk1 = D[k + 1];
            const double ek1 = k < end - 1 ? E[k + 1] : 0.0;
            double c, s;
            make_givens(x, z, c, s);
            const double sdk = s * dk + c * ek;
            const double dkp1 = s * ek + c * dk1;
            const double ndk = c * (c * dk - s * ek) - s * (c * ek - s * dk1);
            const double ndk1 = s * sdk + c * dkp1;
            const double nek = c * sdk - s * dkp1;
            if (lane == 0) {
                D[k] = ndk;
                D[k + 1] = ndk1;
                E[k] = nek;
                if (k > start) E[k - 1] = c * eprev - s * z;
                S.rc[b][k - start] = c;
                S.rs[b][k - start] = s;
            }
            x = nek;
            eprev = nek;
            dk = ndk1;
            if (k < end - 1) {
                z = -s * ek1;
                ek = c * ek1;
                if (lane == 0) E[k + 1] = ek;
            }
        }
        if (lane == 0) {
            S.sw[b][0] = start;
            S.sw[b][1] = k - start;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        return;
    }
}

// Eigen::SelfAdjointEigenSolver<MatrixXd>(A): src column-major (ld lds), lower
// triangle read.  A (n x n, ld n) is the workspace and receives the eigenvectors,
// w the eigenvalues (ascending), hc n doubles of scratch.
__global__ void __launch_bounds__(EIG_THREADS) sym_eigen_kernel(int n, const double* __restrict__ src, int lds,
                                                                double* __restrict__ A, double* __restrict__ w,
                                                                double* __restrict__ hc, int* __restrict__ info) {
    __shared__ EigShared S;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (n == 1) {
        if (tid == 0) {
            w[0] = src[0];
            A[0] = 1.0;
            *info = 0;
        }
        return;
    }
    // ---- scale = max |lower(A)|, mat = lower(A) / scale, kept symmetric
    double mx = 0.0;
    for (int e = tid; e < n * n; e += EIG_THREADS) {
        const int i = e % n, j = e / n;
        if (i >= j) mx = fmax(mx, fabs(src[(long)j * lds + i]));
    }
    mx = wave_max(mx);
    if (lane == 0) S.red[wid] = mx;
    __syncthreads();
    double scale = 0.0;
    for (int k = 0; k < EIG_WAVES; ++k) scale = fmax(scale, S.red[k]);
    if (scale == 0.0) scale = 1.0;
    for (int e = tid; e < n * n; e += EIG_THREADS) {
        const int i = e % n, j = e / n;
        const int hi = i > j ? i : j, lo = i > j ? j : i;
        A[e] = src[(long)lo * lds + hi] / scale;
    }
    __syncthreads();

    // ---- tridiagonalization_inplace.  Every sum runs in the oracle's sequential
    // order (one thread per sum), so the device and oracle/marg.c agree bit for bit.
    for (int i = 0; i < n - 1; ++i) {
        const int rem = n - i - 1, o = i + 1;
        double* col = A + (long)i * n;
        for (int k = tid; k < rem; k += EIG_THREADS) S.v[k] = col[o + k];
        __syncthreads();
        if (tid == 0) {
            double t = 0.0;
            for (int k = 1; k < rem; ++k) t += S.v[k] * S.v[k];
            const double c0 = S.v[0];
            double tau, beta;
            if (t <= DBL_MIN) {
                tau = 0.0;
                beta = c0;
                S.sc[1] = 0.0;  // essential.setZero()
            } else {
                beta = sqrt(c0 * c0 + t);
                if (c0 >= 0.0) beta = -beta;
                tau = (beta - c0) / beta;
                S.sc[1] = c0 - beta;
            }
            S.sc[0] = beta;
            S.red[0] = tau;
        }
        __syncthreads();
        const double h = S.red[0], dv = S.sc[1];
        // essential = tail / (c0 - beta) (or zero), stored in place and in v
        for (int k = 1 + tid; k < rem; k += EIG_THREADS) {
            const double ek = dv == 0.0 ? 0.0 : S.v[k] / dv;
            S.v[k] = ek;
            col[o + k] = ek;
        }
        if (tid == 0) S.v[0] = 1.0;
        __syncthreads();
        // p = A_sub.selfadjointView<Lower>() * (h v): one thread per row, coalesced column walk
        if (tid < rem) {
            const double* a = A + (long)o * n + o + tid;
            double acc = 0.0;
            for (int k = 0; k < rem; ++k, a += n) acc += *a * (h * S.v[k]);
            S.p[tid] = acc;
        }
        __syncthreads();
        if (tid == 0) {
            double d = 0.0;
            for (int k = 0; k < rem; ++k) d += S.p[k] * S.v[k];
            S.sc[1] = (h * -0.5) * d;
        }
        __syncthreads();
        {
            const double sc = S.sc[1];
            for (int k = tid; k < rem; k += EIG_THREADS) S.part[k] = S.p[k] + sc * S.v[k];
        }
        __syncthreads();
        // A_sub -= v p^T + p v^T (rankUpdate, lower formula mirrored)
        for (int e = tid; e < rem * rem; e += EIG_THREADS) {
            const int jj = e % rem, kk = e / rem;
            const int hi = jj > kk ? jj : kk, lo = jj > kk ? kk : jj;
            A[(long)(o + kk) * n + o + jj] += (-S.v[lo]) * S.part[hi] + (-S.part[lo]) * S.v[hi];
        }
        if (tid == 0) {
            col[i + 1] = S.sc[0];
            hc[i] = h;
        }
        __syncthreads();
    }
    for (int i = tid; i < n; i += EIG_THREADS) {
        S.diag[i] = A[(long)i * n + i];
        if (i < n - 1) S.sub[i] = A[(long)i * n + i + 1];
    }
    __syncthreads();

    // ---- Householder sequence evaluated in place (HouseholderSequence::evalTo)
    for (int e = tid; e < n * n; e += EIG_THREADS) {
        const int i = e % n, j = e / n;
        if (i < j) A[e] = 0.0;
        if (i == j) A[e] = 1.0;
    }
    __syncthreads();
    for (int k = n - 2; k >= 0; --k) {
        const int cs = n - k - 1;
        const double tau = hc[k];
        double* C = A + (long)(k + 1) * n + (k + 1);
        if (cs == 1) {
            if (tid == 0) C[0] *= 1.0 - tau;
        } else if (tau != 0.0) {
            const double* ess = A + (long)k * n + k + 2;
            for (int r = tid; r < cs - 1; r += EIG_THREADS) S.v[r] = ess[r];
            __syncthreads();
            // tmp = ess^T * bottom + row0: one thread per column, sequential over rows
            if (tid < cs) {
                const double* cc = C + (long)tid * n;
                double acc = 0.0;
                for (int r = 0; r < cs - 1; ++r) acc += S.v[r] * cc[1 + r];
                S.p[tid] = acc + cc[0];
            }
            __syncthreads();
            for (int e = tid; e < cs * cs; e += EIG_THREADS) {
                const int rr = e % cs, c = e / cs;
                if (rr == 0)
                    C[(long)c * n] -= tau * S.p[c];
                else
                    C[(long)c * n + rr] -= (tau * S.v[rr - 1]) * S.p[c];
            }
        }
        __syncthreads();
        for (int r = k + 1 + tid; r < n; r += EIG_THREADS) A[(long)k * n + r] = 0.0;
    }
    __syncthreads();

    // ---- implicit symmetric QR: wave 0 produces sweeps, waves 1.. apply them to Q's rows
    QrState st{0, n - 1, 0, 0};
    if (wid == 0) qr_produce(S, st, n, 0, lane);
    __syncthreads();
    for (int s = 0;; ++s) {
        const int b = s & 1;
        const int cnt = S.sw[b][1];
        if (cnt < 0) break;
        if (wid == 0) {
            qr_produce(S, st, n, b ^ 1, lane);
        } else {
            const int i = tid - 64;
            if (i < n && cnt > 0) {
                const int k0 = S.sw[b][0];
                double* q = A + i;
                double x = q[(long)k0 * n];
                for (int t = 0; t < cnt; ++t) {
                    const int k = k0 + t;
                    const double c = S.rc[b][t], sn = S.rs[b][t];
                    const double y = q[(long)(k + 1) * n];
                    q[(long)k * n] = c * x - sn * y;
                    x = sn * x + c * y;
                }
                q[(long)(k0 + cnt) * n] = x;
            }
        }
        __syncthreads();
    }
    // ---- selection sort (minCoeff: first index of the minimum), then the column swaps per row
    if (wid == 0) {
        if (st.info == 0) {
            for (int i = 0; i < n - 1; ++i) {
                double best = INFINITY;
                int bi = n;
                for (int j = i + lane; j < n; j += 64) {
                    const double d = S.diag[j];
                    if (d < best) {
                        best = d;
                        bi = j;
                    }
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    const double ob = __shfl_xor(best, o);
                    const int oi = __shfl_xor(bi, o);
                    if (ob < best || (ob == best && oi < bi)) {
                        best = ob;
                        bi = oi;
                    }
                }
                if (lane == 0) {
                    S.swap[i] = bi;
                    if (bi != i) {
                        const double t = S.diag[i];
                        S.diag[i] = S.diag[bi];
                        S.diag[bi] = t;
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
        if (lane == 0) S.sw[0][0] = st.info;
    }
    __syncthreads();
    const int inf = S.sw[0][0];
    if (inf == 0) {
        for (int i = tid; i < n; i += EIG_THREADS) {
            double* q = A + i;
            for (int j = 0; j < n - 1; ++j) {
                const int k = S.swap[j];
                if (k != j) {
                    const double t = q[(long)j * n];
                    q[(long)j * n] = q[(long)k * n];
                    q[(long)k * n] = t;
                }
            }
        }
    }
    for (int i = tid; i < n; i += EIG_THREADS) w[i] = S.diag[i] * scale;
    if (tid == 0) *info = inf;
}

// ------------------------------------------------------------ Schur complement
// Hmm_inv(a, b) = sum_k (V(a, k) d_k) V(b, k), d_k = 1/w_k masked at EPS
__global__ void __launch_bounds__(256) hinv_kernel(int m, const double* __restrict__ V, const double* __restrict__ w,
                                                   double* __restrict__ Hi) {
    const int a = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
    if (a >= m) return;
    double acc = 0.0;
    for (int k = 0; k < m; ++k) {
        const double d = w[k] > MARG_EPS ? 1.0 / w[k] : 0.0;
        acc += (V[(long)k * m + a] * d) * V[(long)k * m + b];
    }
    Hi[(long)b * m + a] = acc;
}

// T = Hrm Hmm_inv (r x m), Hrm = H0(m.., 0..m)
__global__ void __launch_bounds__(256) schur_t_kernel(int L, int m, const double* __restrict__ H0,
                                                      const double* __restrict__ Hi, double* __restrict__ T) {
    const int r = L - m;
    const int a = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
    if (a >= r) return;
    const double* hr = H0 + m + a;
    const double* hi = Hi + (long)b * m;
    double acc = 0.0;
    for (int k = 0; k < m; ++k) acc += hr[(long)k * L] * hi[k];
    T[(long)b * r + a] = acc;
}

// Hp = Hrr - T Hmr (column b < r), bp = brr - T bmm (column b == r)
__global__ void __launch_bounds__(256) schur_p_kernel(int L, int m, const double* __restrict__ H0,
                                                      const double* __restrict__ b0, const double* __restrict__ T,
                                                      double* __restrict__ Hp, double* __restrict__ bp) {
    const int r = L - m;
    const int a = blockIdx.x * 256 + threadIdx.x, b = blockIdx.y;
    if (a >= r) return;
    const double* x = b < r ? H0 + (long)(m + b) * L : b0;  // Hmr column b / bmm
    double acc = 0.0;
    for (int k = 0; k < m; ++k) acc += T[(long)k * r + a] * x[k];
    if (b < r)
        Hp[(long)b * r + a] = H0[(long)(m + b) * L + m + a] - acc;
    else
        bp[a] = b0[m + a] - acc;
}

// J0 = S^1/2 V^T, e0 = (S^-1/2 V^T) (-bp), S masked at EPS
__global__ void __launch_bounds__(256) linearize_kernel(int r, const double* __restrict__ V,
                                                        const double* __restrict__ w, const double* __restrict__ bp,
                                                        double* __restrict__ J0, double* __restrict__ e0) {
    const int i = blockIdx.x * 256 + threadIdx.x, j = blockIdx.y;  // J0(i, j) = sqrt(S_i) V(j, i)
    if (i >= r) return;
    const double wi = w[i];
    const double S = wi > MARG_EPS ? wi : 0.0;
    J0[(long)j * r + i] = sqrt(S) * V[(long)i * r + j];
    if (j == 0) {
        const double sis = sqrt(wi > MARG_EPS ? 1.0 / wi : 0.0);
        const double* v = V + (long)i * r;
        double acc = 0.0;
        for (int k = 0; k < r; ++k) acc += (sis * v[k]) * -bp[k];
        e0[i] = acc;
    }
}

hipError_t launch_eigen(gvx_ctx* c, int n, const double* src, int lds, double* V, double* w, double* hc, int* info) {
    if (n <= 0) return hipSuccess;
    sym_eigen_kernel<<<1, EIG_THREADS, 0, c->stream>>>(n, src, lds, V, w, hc, info);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_sym_eigen(gvx_ctx* c, int n, const double* src, int lds, double* V, double* w, double* hc,
                            int* info) {
    return launch_eigen(c, n, src, lds, V, w, hc, info);
}

hipError_t launch_marginalize(gvx_ctx* c, const MargLaunch& p) {
    const int r = p.L - p.m;
    hipError_t e = hipMemsetAsync(p.H0, 0, sizeof(double) * (size_t)p.L * p.L, c->stream);
    if (e != hipSuccess) return e;
    if (p.loss) {
        loss_kernel<<<(p.n_fac + 63) / 64, 64, 0, c->stream>>>(p.n_fac, p.nres, p.res_off, p.loss, p.data, p.sr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (p.n_pairs + p.n_bvec > 0) {
        h0_kernel<<<p.n_pairs + p.n_bvec, H0_THREADS, 0, c->stream>>>(p.n_pairs, p.pairs, p.contrib, p.data,
                                                                       p.loss ? p.sr : nullptr, p.L, p.H0, p.b0);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    // Hmm = 0.5 (H0mm + H0mm^T) is H0mm itself: h0_kernel writes both triangles alike
    if ((e = launch_eigen(c, p.m, p.H0, p.L, p.V1, p.w1, p.hc, p.info)) != hipSuccess) return e;
    if (p.m > 0) {
        hinv_kernel<<<dim3((p.m + 255) / 256, p.m), 256, 0, c->stream>>>(p.m, p.V1, p.w1, p.Hinv);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (r <= 0) return hipSuccess;
    if (p.m > 0) {
        schur_t_kernel<<<dim3((r + 255) / 256, p.m), 256, 0, c->stream>>>(p.L, p.m, p.H0, p.Hinv, p.T);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    schur_p_kernel<<<dim3((r + 255) / 256, r + 1), 256, 0, c->stream>>>(p.L, p.m, p.H0, p.b0, p.T, p.Hp, p.bp);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = launch_eigen(c, r, p.Hp, r, p.V2, p.w2, p.hc, p.info + 1)) != hipSuccess) return e;
    linearize_kernel<<<dim3((r + 255) / 256, r), 256, 0, c->stream>>>(r, p.V2, p.w2, p.bp, p.J0, p.e0);
    return hipGetLastError();
}

}  // namespace gvx
