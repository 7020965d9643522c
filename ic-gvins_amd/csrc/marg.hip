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
//   wave 0 runs the scalar Givens chain of sweep s+1 while 12 waves (not those on
//   wave 0's SIMD) apply the rotations of sweep s to the rows of Q (a row's
//   rotations need no other row, so a sweep costs one barrier), and finally the
//   selection sort.
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

// the restatement's sum64 fold (oracle/marg.c): lane l holds the partial sum of
// elements l, l + 64, ...; the xor butterfly leaves the total in every lane
__device__ inline double bfly_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = v + __shfl_xor(v, o);
    return v;
}

// column chunks of the tridiagonalisation mat-vec (oracle/marg.c eig_groups)
__device__ inline int eig_groups(int rem) {
    const int rpad = (rem + 63) & ~63;
    const int g = 1024 / rpad;
    return g > 16 ? 16 : g;
}

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

// The same sums split into chunks of a record's contribution list (the FAST
// path: the extrinsic and td pairs of a window carry every reprojection factor,
// 1,800 contributions that h0_kernel walks in one thread each): one workgroup
// per chunk writes its partial sums, then h0_sum_kernel adds a record's partials
// in chunk order.
__global__ void __launch_bounds__(H0_THREADS) h0_part_kernel(int n_pairs, const MargPairRec* __restrict__ pairs,
                                                             const int4* __restrict__ chunks,
                                                             const int4* __restrict__ contrib,
                                                             const double* __restrict__ data,
                                                             const double* __restrict__ sr,
                                                             double* __restrict__ part) {
    const int4 ch = chunks[blockIdx.x];
    const MargPairRec pr = pairs[ch.x];
    const bool hrec = ch.x < n_pairs;
    const int n_ent = pr.lp * pr.lq;
    for (int e = threadIdx.x; e < n_ent; e += H0_THREADS) {
        const int a = e % pr.lp, b = e / pr.lp;
        double h = 0.0;
        for (int ci = ch.y; ci < ch.z; ++ci) {
            const int4 c = contrib[ci];
            const int gp = c.z & 255, gq = (c.z >> 8) & 255, nres = c.z >> 16;
            const double s = sr ? sr[c.w] : 1.0;
            const double* jp = data + c.x + a;
            const double* jq = data + c.y + (hrec ? b : 0);
            double acc = 0.0;
            for (int r = 0; r < nres; ++r) acc += (s * jp[(long)r * gp]) * (s * jq[(long)r * gq]);
            if (hrec)
                h += acc;
            else
                h -= acc;
        }
        part[ch.w + e] = h;
    }
}

__global__ void __launch_bounds__(H0_THREADS) h0_sum_kernel(int n_pairs, const MargPairRec* __restrict__ pairs,
                                                            const int2* __restrict__ recpart,
                                                            const double* __restrict__ part, int L,
                                                            double* __restrict__ H0, double* __restrict__ b0) {
    const MargPairRec pr = pairs[blockIdx.x];
    const int2 rp = recpart[blockIdx.x];
    const int n_ent = pr.lp * pr.lq;
    for (int e = threadIdx.x; e < n_ent; e += H0_THREADS) {
        const int a = e % pr.lp, b = e / pr.lp;
        double h = part[rp.x + e];
        for (int k = 1; k < rp.y; ++k) h += part[rp.x + k * n_ent + e];
        if ((int)blockIdx.x < n_pairs) {
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
    long rot;  // rotations produced (diagnostics)
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
        st.rot += k - start;
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
                                                                double* __restrict__ hc, int* __restrict__ info,
                                                                unsigned long long* __restrict__ ts,
                                                                const int* __restrict__ run_if) {
    __shared__ EigShared S;
    if (run_if && *run_if == 0) return;  // the Cholesky path (dense.hip) succeeded
    // ts (nullable, diagnostics): wall clock (100 MHz) at the phase boundaries
#define EIG_STAMP(k) \
    if (ts && tid == 0) ts[k] = wall_clock64()
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    EIG_STAMP(0);
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

    EIG_STAMP(1);
    // ---- tridiagonalization_inplace.  Sums use the restatement's fixed orders
    // (oracle/marg.c: sum64 = 64 lane-strided partial sums folded by an xor
    // butterfly; the mat-vec = G column chunks folded in order), so the device
    // and the restatement agree bit for bit.
    for (int i = 0; i < n - 1; ++i) {
        const int rem = n - i - 1, o = i + 1;
        double* col = A + (long)i * n;
        if (wid == 0) {
            // makeHouseholderInPlace on v = col[i+1 ..)
            double t = 0.0;
            for (int k = 1 + lane; k < rem; k += 64) {
                const double x = col[o + k];
                S.v[k] = x;
                t += x * x;
            }
            t = bfly_sum(t);
            const double c0 = col[o];
            double tau, beta, d = 0.0;
            if (t <= DBL_MIN) {
                tau = 0.0;
                beta = c0;
            } else {
                beta = sqrt(c0 * c0 + t);
                if (c0 >= 0.0) beta = -beta;
                tau = (beta - c0) / beta;
                d = c0 - beta;
            }
            for (int k = 1 + lane; k < rem; k += 64) {
                const double ek = d == 0.0 ? 0.0 : S.v[k] / d;  // tail / (c0 - beta), or setZero()
                S.v[k] = ek;
                col[o + k] = ek;
            }
            if (lane == 0) {
                S.v[0] = 1.0;
                S.sc[0] = beta;
                S.sc[1] = tau;
            }
        }
        __syncthreads();
        const double h = S.sc[1];
        // p = A_sub.selfadjointView<Lower>() * (h v): rows over lanes (coalesced
        // column walks), G chunks of columns over the thread groups
        const int G = eig_groups(rem), chunk = (rem + G - 1) / G, rpad = (rem + 63) & ~63;
        {
            const int j = tid % rpad, g = tid / rpad;
            if (g < G && j < rem) {
                const int k0 = g * chunk, k1 = min(rem, k0 + chunk);
                const double* a = A + (long)(o + k0) * n + o + j;
                double acc = 0.0;
                int k = k0;
                for (; k + 8 <= k1; k += 8, a += 8 * (long)n) {
                    double x[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) x[u] = a[(long)u * n];
#pragma unroll
                    for (int u = 0; u < 8; ++u) acc += x[u] * (h * S.v[k + u]);
                }
                for (; k < k1; ++k, a += n) acc += *a * (h * S.v[k]);
                S.part[g * rpad + j] = acc;
            }
        }
        __syncthreads();
        if (wid == 0) {
            double dt = 0.0;
            for (int j = lane; j < rem; j += 64) {
                double s = 0.0;
                for (int g = 0; g < G; ++g) s += S.part[g * rpad + j];
                S.p[j] = s;
                dt += s * S.v[j];
            }
            dt = bfly_sum(dt);
            if (lane == 0) {
                S.sc[1] = (h * -0.5) * dt;
                col[o] = S.sc[0];  // the subdiagonal: beta
                hc[i] = h;
            }
        }
        __syncthreads();
        // A_sub -= v p'^T + p' v^T, p' = p + sc v (rankUpdate, lower formula mirrored):
        // lanes over the rows, 2 columns per wave per batch with every load issued
        // before the first store (the matrix lives in L2: latency, not bandwidth)
        {
            const double sc = S.sc[1];
            const int nr = (rem + 63) >> 6;  // row slots per lane (<= 8)
            for (int k0 = wid * 2; k0 < rem; k0 += 2 * EIG_WAVES) {
                double x[2][8];
#pragma unroll
                for (int cc = 0; cc < 2; ++cc) {
                    const double* ac = A + (long)(o + k0 + cc) * n + o;
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int jj = lane + 64 * u;
                        if (u < nr && k0 + cc < rem && jj < rem) x[cc][u] = ac[jj];
                    }
                }
#pragma unroll
                for (int cc = 0; cc < 2; ++cc) {
                    const int kk = k0 + cc;
                    double* ac = A + (long)(o + kk) * n + o;
                    const double vk = S.v[kk], pk = S.p[kk] + sc * vk;
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int jj = lane + 64 * u;
                        if (u < nr && jj < rem && kk < rem) {
                            const double vj = S.v[jj], pj = S.p[jj] + sc * vj;
                            // lower formula of element (hi, lo): (-v_lo) p'_hi + (-p'_lo) v_hi
                            ac[jj] = x[cc][u] + (jj >= kk ? (-vk) * pj + (-pk) * vj : (-vj) * pk + (-pj) * vk);
                        }
                    }
                }
            }
        }
        __syncthreads();
    }
    for (int i = tid; i < n; i += EIG_THREADS) {
        S.diag[i] = A[(long)i * n + i];
        if (i < n - 1) S.sub[i] = A[(long)i * n + i + 1];
    }
    __syncthreads();

    EIG_STAMP(2);
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
        const double* ess = A + (long)k * n + k + 2;  // cs - 1 entries
        if (cs == 1) {
            if (tid == 0) C[0] *= 1.0 - tau;
        } else if (tau != 0.0) {
            // tmp = ess^T * bottom + row0: one wave per column, sum64 over the rows
            for (int c0 = wid * 2; c0 < cs; c0 += 2 * EIG_WAVES) {
                double acc[2] = {0.0, 0.0};
                const int c1 = min(c0 + 1, cs - 1);
                for (int r = lane; r < cs - 1; r += 64) {
                    const double er = ess[r];
                    acc[0] += er * C[(long)c0 * n + 1 + r];
                    acc[1] += er * C[(long)c1 * n + 1 + r];
                }
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const double t = bfly_sum(acc[q]);
                    if (lane == 0 && c0 + q < cs) S.p[c0 + q] = t + C[(long)(c0 + q) * n];
                }
            }
            __syncthreads();
            const int nr = (cs + 63) >> 6;
            double f[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int rr = lane + 64 * u;
                f[u] = (u < nr && rr < cs) ? (rr == 0 ? tau : tau * ess[rr - 1]) : 0.0;
            }
            for (int c0 = wid * 2; c0 < cs; c0 += 2 * EIG_WAVES) {
                double x[2][8];
#pragma unroll
                for (int q = 0; q < 2; ++q)
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int rr = lane + 64 * u;
                        if (u < nr && c0 + q < cs && rr < cs) x[q][u] = C[(long)(c0 + q) * n + rr];
                    }
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const double tc = S.p[min(c0 + q, cs - 1)];
                    double* cc = C + (long)(c0 + q) * n;
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int rr = lane + 64 * u;
                        if (u < nr && rr < cs && c0 + q < cs) cc[rr] = x[q][u] - f[u] * tc;
                    }
                }
            }
        }
        __syncthreads();
        for (int r = k + 1 + tid; r < n; r += EIG_THREADS) A[(long)k * n + r] = 0.0;
    }
    __syncthreads();

    EIG_STAMP(3);
    // ---- implicit symmetric QR: wave 0 produces sweeps, waves 1.. apply them to Q's rows
    QrState st{0, n - 1, 0, 0, 0};
    if (wid == 0) qr_produce(S, st, n, 0, lane);
    __syncthreads();
    for (int s = 0;; ++s) {
        const int b = s & 1;
        const int cnt = S.sw[b][1];
        if (cnt < 0) break;
        if (wid == 0) {
            qr_produce(S, st, n, b ^ 1, lane);
        } else if (wid & 3) {
            // waves 4, 8, 12 share wave 0's SIMD (round-robin placement): they stay
            // idle so the dependent Givens chain has that SIMD to itself
            const int i = (wid - 1 - (wid >> 2)) * 64 + lane;
            if (i < n && cnt > 0) {
                // Q = Q G_k for k = k0 .. k0+cnt-1 on row i; the row's columns are
                // loaded 8 ahead so the L2 latency is paid once per 8 rotations
                const int k0 = S.sw[b][0];
                double* q = A + i + (long)k0 * n;
                double x = q[0];
                int t = 0;
                for (; t + 8 <= cnt; t += 8, q += 8 * (long)n) {
                    double y[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) y[u] = q[(long)(u + 1) * n];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const double c = S.rc[b][t + u], sn = S.rs[b][t + u];
                        q[(long)u * n] = c * x - sn * y[u];
                        x = sn * x + c * y[u];
                    }
                }
                for (; t < cnt; ++t, q += n) {
                    const double c = S.rc[b][t], sn = S.rs[b][t];
                    const double y = q[n];
                    q[0] = c * x - sn * y;
                    x = sn * x + c * y;
                }
                q[0] = x;
            }
        }
        __syncthreads();
    }
    EIG_STAMP(4);
    if (ts && tid == 0) ts[6] = st.iter;
    if (ts && tid == 0) ts[7] = st.rot;
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
    EIG_STAMP(5);
#undef EIG_STAMP
}

// ------------------------------------------------------------ Schur complement
// Hmm_inv(a, b) = sum_k (V(a, k) d_k) V(b, k), d_k = 1/w_k masked at EPS
// run_if (nullable): the eigen-solver path only runs where the Cholesky path's
// check failed (*run_if != 0)
__global__ void __launch_bounds__(256) hinv_kernel(int m, const double* __restrict__ V, const double* __restrict__ w,
                                                   double* __restrict__ Hi, const int* __restrict__ run_if) {
    if (run_if && *run_if == 0) return;
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
                                                      const double* __restrict__ Hi, double* __restrict__ T,
                                                      const int* __restrict__ run_if) {
    if (run_if && *run_if == 0) return;
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
                                                      double* __restrict__ Hp, double* __restrict__ bp,
                                                      const int* __restrict__ run_if) {
    if (run_if && *run_if == 0) return;
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
                                                        double* __restrict__ J0, double* __restrict__ e0,
                                                        const int* __restrict__ run_if) {
    if (run_if && *run_if == 0) return;
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

hipError_t launch_eigen(gvx_ctx* c, int n, const double* src, int lds, double* V, double* w, double* hc, int* info,
                        unsigned long long* ts = nullptr, const int* run_if = nullptr) {
    if (n <= 0) return hipSuccess;
    sym_eigen_kernel<<<1, EIG_THREADS, 0, c->stream>>>(n, src, lds, V, w, hc, info, ts, run_if);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_sym_eigen(gvx_ctx* c, int n, const double* src, int lds, double* V, double* w, double* hc,
                            int* info, unsigned long long* ts) {
    return launch_eigen(c, n, src, lds, V, w, hc, info, ts);
}

hipError_t launch_h0(gvx_ctx* c, const MargLaunch& p) {
    hipError_t e = hipMemsetAsync(p.H0, 0, sizeof(double) * (size_t)p.L * p.L, c->stream);
    if (e != hipSuccess) return e;
    if (p.loss) {
        loss_kernel<<<(p.n_fac + 63) / 64, 64, 0, c->stream>>>(p.n_fac, p.nres, p.res_off, p.loss, p.data, p.sr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (p.n_pairs + p.n_bvec <= 0) return hipSuccess;
    if (p.chunks && p.n_chunks > 0) {
        h0_part_kernel<<<p.n_chunks, H0_THREADS, 0, c->stream>>>(p.n_pairs, p.pairs, p.chunks, p.contrib, p.data,
                                                                 p.loss ? p.sr : nullptr, p.part);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        h0_sum_kernel<<<p.n_pairs + p.n_bvec, H0_THREADS, 0, c->stream>>>(p.n_pairs, p.pairs, p.recpart, p.part,
                                                                           p.L, p.H0, p.b0);
        return hipGetLastError();
    }
    h0_kernel<<<p.n_pairs + p.n_bvec, H0_THREADS, 0, c->stream>>>(p.n_pairs, p.pairs, p.contrib, p.data,
                                                                   p.loss ? p.sr : nullptr, p.L, p.H0, p.b0);
    return hipGetLastError();
}

hipError_t launch_marginalize(gvx_ctx* c, const MargLaunch& p) {
    const int r = p.L - p.m;
    const bool fast = p.solver == GVX_MARG_SOLVER_FAST;
    hipError_t e = launch_h0(c, p);
    if (e != hipSuccess) return e;
    // FAST: Cholesky path where Hmm - EPS*I (then Hp - EPS*I) is positive definite
    // (dense.hip), the eigen-solver path below only where that check failed;
    // chol[k] != 0 marks the failure, read by the kernels on the device
    const int* gate_m = fast ? p.chol : nullptr;
    const int* gate_r = fast ? p.chol + 1 : nullptr;
    if (fast && p.m > 0) {
        if ((e = launch_potrf(c, p.m, p.H0, p.L, MARG_EPS, p.Lm, p.chol, nullptr)) != hipSuccess) return e;
        if ((e = launch_potrf(c, p.m, p.H0, p.L, 0.0, p.Lm, p.chol, p.chol)) != hipSuccess) return e;
    }
    // Hmm = 0.5 (H0mm + H0mm^T) is H0mm itself: h0_kernel writes both triangles alike
    if ((e = launch_eigen(c, p.m, p.H0, p.L, p.V1, p.w1, p.hc, p.info, nullptr, gate_m)) != hipSuccess) return e;
    if (p.m > 0) {
        hinv_kernel<<<dim3((p.m + 255) / 256, p.m), 256, 0, c->stream>>>(p.m, p.V1, p.w1, p.Hinv, gate_m);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (r <= 0) return hipSuccess;
    if (p.m > 0) {
        schur_t_kernel<<<dim3((r + 255) / 256, p.m), 256, 0, c->stream>>>(p.L, p.m, p.H0, p.Hinv, p.T, gate_m);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    schur_p_kernel<<<dim3((r + 255) / 256, r + 1), 256, 0, c->stream>>>(p.L, p.m, p.H0, p.b0, p.T, p.Hp, p.bp,
                                                                         gate_m);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (fast) {
        if (p.m > 0) {
            // X = Lm^-1 [Hmr | bm] (row-major m x (r + 1)), then Hp, bp
            if ((e = launch_trsv(c, p.m, p.Lm, r, p.H0 + (size_t)p.m * p.L, p.L, p.X, r + 1, false, p.chol)) !=
                hipSuccess)
                return e;
            if ((e = launch_trsv(c, p.m, p.Lm, 1, p.b0, p.m, p.X + r, r + 1, false, p.chol)) != hipSuccess) return e;
            if ((e = launch_schur_chol(c, p.L, p.m, p.H0, p.b0, p.X, p.Hp, p.bp, p.chol)) != hipSuccess) return e;
        }
        if ((e = launch_potrf(c, r, p.Hp, r, MARG_EPS, p.Lp, p.chol + 1, nullptr)) != hipSuccess) return e;
        if ((e = launch_potrf(c, r, p.Hp, r, 0.0, p.Lp, p.chol + 1, p.chol + 1)) != hipSuccess) return e;
    }
    if ((e = launch_eigen(c, r, p.Hp, r, p.V2, p.w2, p.hc, p.info + 1, nullptr, gate_r)) != hipSuccess) return e;
    linearize_kernel<<<dim3((r + 255) / 256, r), 256, 0, c->stream>>>(r, p.V2, p.w2, p.bp, p.J0, p.e0, gate_r);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (fast) {
        // J0 = Lp^T, e0 = -Lp^-1 bp
        if ((e = launch_lin_chol(c, r, p.Lp, p.J0, p.w2, p.chol + 1)) != hipSuccess) return e;
        if ((e = launch_trsv(c, r, p.Lp, 1, p.bp, r, p.e0, 1, true, p.chol + 1)) != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace gvx
