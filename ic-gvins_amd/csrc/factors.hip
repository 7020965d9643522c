// factors.hip -- batched residual + Jacobian evaluation of the two BA factor
// types on gfx950 (fp64):
//   ReprojectionFactor::Evaluate    factors/reprojection_factor.h:61-161
//   PreintegrationFactor::Evaluate  preintegration/preintegration_factor.h:45-69
//     -> Preintegration{Normal,Earth}::evaluate + residualJacobian{Pose,Mix}{0,1}
// (paths under /root/reference/ic_gvins/ic_gvins/).
//
// Reprojection: one lane per factor; parameter blocks are gathered through the
// per-factor offset table (the Ceres parameter-block pointers), outputs are
// staged through LDS so that the 46-double Jacobian rows leave as coalesced
// stores.  Preintegration: 16 lanes per factor (preint_factor_kernel), the
// whitening on the fp64 matrix cores; the
// reference's per-call sqrt_information_ = LLT(P^-1)^T (quirk, SURVEY.md App.
// C.2) is formed once per segment by sqrt_info_kernel with the same arithmetic.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdlib>

#include "dmath.h"
#include "gvx_internal.h"

namespace gvx {

namespace {

constexpr int NS = 15;

// ------------------------------------------------------------ reprojection
// C(2x3) = A(2x3) * B(3x3)
__device__ __forceinline__ void m23m33(const double* A, const double* B, double* C) {
    double t[6];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 3; ++j)
            t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
    for (int k = 0; k < 6; ++k) C[k] = t[k];
}

__device__ __forceinline__ void put_2x7(const double* red, const double* L, const double* R, double* J) {
    double a[6], b[6];
    m23m33(red, L, a);
    m23m33(red, R, b);
    for (int i = 0; i < 2; ++i) {
        for (int j = 0; j < 3; ++j) {
            J[7 * i + j] = a[3 * i + j];
            J[7 * i + 3 + j] = b[3 * i + j];
        }
        J[7 * i + 6] = 0.0;
    }
}

constexpr int RP_THREADS = 128;
constexpr int RP_OUT = 48;  // residual 2 + Jacobians 46

constexpr int RP_LDS = RP_THREADS * (RP_OUT + 1);  // doubles of the output staging
// block `blk` of the reprojection batch (RP_THREADS threads): the body of
// reproj_kernel and of window_factor_kernel's reprojection blocks
__device__ __forceinline__ void reproj_body(int blk, double* __restrict__ stage, int n,
                                            const gvx_reproj_const* __restrict__ cs,
                                            const double* __restrict__ params, const int32_t* __restrict__ offs,
                                            double* __restrict__ res, double* __restrict__ jac) {
    const int t = threadIdx.x;
    const int base = blk * RP_THREADS;
    const int i = base + t;
    double* out = stage + t * (RP_OUT + 1);
    if (i < n) {
        const gvx_reproj_const c = cs[i];
        const int32_t* o = offs + 5 * (int64_t)i;
        const double* P0 = params + o[0];
        const double* P1 = params + o[1];
        const double* EX = params + o[2];
        const dq q0 = dq_make(P0[6], P0[3], P0[4], P0[5]);
        const dq q1 = dq_make(P1[6], P1[3], P1[4], P1[5]);
        const dq qic = dq_make(EX[6], EX[3], EX[4], EX[5]);
        const double p0[3] = {P0[0], P0[1], P0[2]}, p1[3] = {P1[0], P1[1], P1[2]};
        const double tic[3] = {EX[0], EX[1], EX[2]};
        const double id0 = params[o[3]];
        const double td = params[o[4]];
        const double sq = 1.0 / c.std;
        const double SI[4] = {sq, 0.0, 0.0, sq};
        double pts0td[3], pts1td[3], pc0[3], pb0[3], pn[3], pb1[3], pts1[3], tv[3];
        for (int k = 0; k < 3; ++k) {
            pts0td[k] = c.pts0[k] - (td - c.td0) * c.vel0[k];
            pts1td[k] = c.pts1[k] - (td - c.td1) * c.vel1[k];
        }
        for (int k = 0; k < 3; ++k) pc0[k] = pts0td[k] / id0;
        dq_rotate(qic, pc0, tv);
        for (int k = 0; k < 3; ++k) pb0[k] = tv[k] + tic[k];
        dq_rotate(q0, pb0, tv);
        for (int k = 0; k < 3; ++k) pn[k] = tv[k] + p0[k];
        for (int k = 0; k < 3; ++k) tv[k] = pn[k] - p1[k];
        dq_rotate(dq_inv(q1), tv, pb1);
        for (int k = 0; k < 3; ++k) tv[k] = pb1[k] - tic[k];
        dq_rotate(dq_inv(qic), tv, pts1);
        const double d1 = pts1[2];
        const double e0 = pts1[0] / d1 - pts1td[0];
        const double e1 = pts1[1] / d1 - pts1td[1];
        out[0] = SI[0] * e0 + SI[1] * e1;
        out[1] = SI[2] * e0 + SI[3] * e1;
        if (jac) {
            double cb0n[9], cnb1[9], cbc[9], R[9];
            dq_rot(q0, cb0n);
            dq_rot(q1, R);
            mt3(R, cnb1);
            dq_rot(qic, R);
            mt3(R, cbc);
            const double red0[6] = {1.0 / d1, 0, -pts1[0] / (d1 * d1), 0, 1.0 / d1, -pts1[1] / (d1 * d1)};
            double red[6];
            for (int a = 0; a < 2; ++a)
                for (int b = 0; b < 3; ++b) red[3 * a + b] = SI[2 * a] * red0[b] + SI[2 * a + 1] * red0[3 + b];
            double A[9], B[9], C[9], S[9];
            // A = cbc*cnb1 and AC = A*cb0n are shared: J0 = [A | (-AC) S(pb0)],
            // J1 = [-A | ...], J2's tmp_r = AC cbc^T (the restatement forms them
            // separately; negation is exact, so the bits are the same)
            double AC[9], nA[9];
            mm3(cbc, cnb1, A);
            mm3(A, cb0n, AC);
            for (int k = 0; k < 9; ++k) {
                nA[k] = -A[k];
                B[k] = -AC[k];
            }
            // J0: pose_i
            skew(pb0, S);
            mm3(B, S, B);
            put_2x7(red, A, B, out + 2);
            // J1: pose_j
            skew(pb1, S);
            mm3(cbc, S, B);
            put_2x7(red, nA, B, out + 16);
            // J2: extrinsic
            mm3(cnb1, cb0n, C);
            for (int k = 0; k < 9; ++k) C[k] = C[k] - ((k % 4) == 0 ? 1.0 : 0.0);
            mm3(cbc, C, A);
            double tmp_r[9], cbcT[9], ntr[9], S1[9], S2[9], S3[9], u[3], w[3];
            mt3(cbc, cbcT);
            mm3(AC, cbcT, tmp_r);
            for (int k = 0; k < 9; ++k) ntr[k] = -tmp_r[k];
            skew(pc0, S);
            mm3(ntr, S, S1);
            mv3(tmp_r, pc0, u);
            skew(u, S2);
            mv3(cb0n, tic, u);
            for (int k = 0; k < 3; ++k) u[k] = u[k] + p0[k] - p1[k];
            mv3(cnb1, u, w);
            for (int k = 0; k < 3; ++k) w[k] = w[k] - tic[k];
            mv3(cbc, w, u);
            skew(u, S3);
            for (int k = 0; k < 9; ++k) B[k] = S1[k] + S2[k] + S3[k];
            put_2x7(red, A, B, out + 30);
            // J3: inverse depth, J4: td
            double nred[6], M[6], v2[2];
            for (int k = 0; k < 6; ++k) nred[k] = -red[k];
            m23m33(nred, cbc, M);
            m23m33(M, cnb1, M);
            m23m33(M, cb0n, M);
            m23m33(M, cbcT, M);
            v2[0] = M[0] * pts0td[0] + M[1] * pts0td[1] + M[2] * pts0td[2];
            v2[1] = M[3] * pts0td[0] + M[4] * pts0td[1] + M[5] * pts0td[2];
            const double dd = id0 * id0;
            out[44] = v2[0] / dd;
            out[45] = v2[1] / dd;
            v2[0] = M[0] * c.vel0[0] + M[1] * c.vel0[1] + M[2] * c.vel0[2];
            v2[1] = M[3] * c.vel0[0] + M[4] * c.vel0[1] + M[5] * c.vel0[2];
            const double s0 = SI[0] * c.vel1[0] + SI[1] * c.vel1[1];
            const double s1 = SI[2] * c.vel1[0] + SI[3] * c.vel1[1];
            out[46] = v2[0] / id0 + s0;
            out[47] = v2[1] / id0 + s1;
        }
    }
    __syncthreads();
    // coalesced write-out of the block's residuals and Jacobians
    const int cnt = min(RP_THREADS, n - base);
    for (int k = t; k < cnt * 2; k += RP_THREADS) {
        const int f = k >> 1, q = k & 1;
        __builtin_nontemporal_store(stage[f * (RP_OUT + 1) + q], res + (int64_t)base * 2 + k);
    }
    if (jac)
        for (int k = t; k < cnt * 46; k += RP_THREADS) {
            const int f = k / 46, q = k - f * 46;
            __builtin_nontemporal_store(stage[f * (RP_OUT + 1) + 2 + q], jac + (int64_t)base * 46 + k);
        }
}

__global__ void __launch_bounds__(RP_THREADS) reproj_kernel(int n, const gvx_reproj_const* __restrict__ cs,
                                                             const double* __restrict__ params,
                                                             const int32_t* __restrict__ offs,
                                                             double* __restrict__ res,
                                                             double* __restrict__ jac) {
    __shared__ double stage[RP_LDS];
    reproj_body(blockIdx.x, stage, n, cs, params, offs, res, jac);
}

// ------------------------------------------------------ preintegration factor
__device__ __forceinline__ void set3(double* J, int ld, int r, int c, const double* B) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) J[(r + i) * ld + c + j] = B[3 * i + j];
}

// sqrt_information_ = LLT(covariance_.inverse()).matrixL().transpose()
// (preintegration_earth.cc:39-40; the Normal variant likewise) for factor
// sets and integrate calls that do not run preint_cov16_kernel (which forms it
// in its epilogue): four segments per wavefront, 16 lanes each (the per-step
// scalar work -- pivot search, divisions, the LLT's dot products -- issued once
// for four segments), by dmath.h sqrt_info_group.  The reference recomputes
// the factor inside every Evaluate; it depends on covariance_ alone, so it is
// formed once here with the same arithmetic and stored upper triangular in
// gvx_preint_result::sqrt_info.
constexpr int SQ_SEG = 4;  // segments per 64-lane workgroup
__global__ void __launch_bounds__(64) sqrt_info_kernel(int n, gvx_preint_result* __restrict__ pre) {
    __shared__ double As[SQ_SEG][NS * NS];  // LU
    __shared__ double Xs[SQ_SEG][NS * NS];  // inverse, then Cholesky factor
    __shared__ int perms[SQ_SEG][NS];
    const int g = threadIdx.x >> 4, gl = threadIdx.x & 15;
    const int fi = blockIdx.x * SQ_SEG + g;
    const bool live = fi < n;  // a spare group factors the identity
    gvx_preint_result* s = pre + (live ? fi : 0);
    for (int e = gl; e < NS * NS; e += 16) As[g][e] = live ? s->covariance[e] : (e % (NS + 1) == 0 ? 1.0 : 0.0);
    sqrt_info_group(As[g], Xs[g], perms[g], gl, live ? s->sqrt_info : nullptr);
}

// One factor per 16-lane group, 4 factors per 64-lane workgroup (one wave).
// Every input is staged into LDS before any of it is used, in two dependent
// rounds of loads and no more: round 1 (issued first, needing only the factor
// index) brings each factor's record -- sqrt_info's upper triangle, the 9 x 6
// bias block of jacobian_, the delta state, gravity and iewn -- through
// global_load_lds (4 bytes a lane, any source address, no registers), plus the
// per-factor offsets and pn_ extents; round 2 brings the four parameter blocks
// into the record and the first 128 pn_ samples into the 16 KB tile region.
// (r02's form loaded the same data where it was used: five to six dependent
// memory round trips per wave, half of its 61 k cycles spent waiting.)
// The residual and the raw Jacobian blocks are uniform per factor: the group's
// lanes compute them together (one instruction stream for the wave's four
// factors) and lane 0 of the group stores them into the group's LDS tile
// Jr[15][33] (32 Jacobian columns [J0 7 | J1 9 | J2 7 | J3 9] + the residual).
// Earth: the position-correction sum over pn_ runs on all 16 lanes of the
// group (a strided partial sum each, then a DPP butterfly), from the staged
// samples.
// Whitening sqrt_info * [Jr | r] runs on the matrix cores (v_mfma_f64_16x16x4,
// 12 per factor); the wave then stores its four factors' residuals and
// Jacobians as contiguous runs.
#ifndef PF_LANES
#define PF_LANES 16
#endif
constexpr int PF_L = PF_LANES;           // lanes per factor (>= 3: the p_cor components)
constexpr int PF_GROUPS = 64 / PF_L;     // factors per workgroup (one wave)
constexpr int PF_SLOTS = (64 + PF_L - 1) / PF_L;  // groups incl. a partial one (idle lanes)
constexpr int PF_LD = 33;                // tile row: 32 Jacobian columns + the residual
constexpr int PN_CH = 64;                // pn_ samples per factor per LDS chunk
constexpr int PN_PER = PF_L / 2;         // samples per factor per global_load_lds (16 B per lane)
constexpr int PN_INS = PN_CH / PN_PER;   // instructions per chunk (1 KB each)
// the factor record in LDS (doubles): sqrt_info upper triangle (row-major,
// packed), jacobian_ rows 0..8 x columns 9..14, misc, the four parameter blocks
constexpr int RC_SQ = 0, RC_J6 = 120, RC_MISC = 174, RC_PAR = 197, RC_N = 229, RC_STRIDE = 256;
// misc: delta_time, then delta.p, .q, .v, .bg, .ba, gravity, iewn (contiguous in the struct)
constexpr int RC_DT = RC_MISC, RC_DP = RC_MISC + 1, RC_DQ = RC_MISC + 4, RC_DV = RC_MISC + 8,
              RC_DBG = RC_MISC + 11, RC_DBA = RC_MISC + 14, RC_G = RC_MISC + 17, RC_IEWN = RC_MISC + 20;
static_assert(offsetof(gvx_preint_result, gravity) == offsetof(gvx_preint_result, delta) + sizeof(gvx_state) &&
                  offsetof(gvx_preint_result, iewn) == offsetof(gvx_preint_result, gravity) + 24 &&
                  offsetof(gvx_state, p) == 8 && offsetof(gvx_state, q) == 32 && offsetof(gvx_state, v) == 64 &&
                  offsetof(gvx_state, bg) == 88 && offsetof(gvx_state, ba) == 112,
              "the misc block is one contiguous run of the struct");
static_assert(RC_PAR == RC_MISC + 23 && RC_N == RC_PAR + 32 && RC_N <= RC_STRIDE, "record layout");
static_assert(RC_DQ - RC_DP == 3 && RC_DV - RC_DQ == 4 && RC_DBG - RC_DV == 3 && RC_DBA - RC_DBG == 3 &&
                  RC_G - RC_DBA == 3 && RC_IEWN - RC_G == 3,
              "misc mirrors delta.{p, q, v, bg, ba}, gravity, iewn");

// v of the lane n places down its 16-lane row, cyclically (DPP row_ror:n), fp64
template <int N>
__device__ __forceinline__ double dpp_row_ror(double v) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    return __hiloint2double(__builtin_amdgcn_update_dpp(0, hi, 0x120 + N, 0xf, 0xf, false),
                            __builtin_amdgcn_update_dpp(0, lo, 0x120 + N, 0xf, 0xf, false));
}

// packed upper-triangular index of (r, c), c >= r, n = 15
__device__ __forceinline__ int triu15(int r, int c) { return r * 15 - (r * (r - 1)) / 2 + (c - r); }

constexpr int PF_TILE = 2 * PN_INS * 128;        // doubles: pn_ chunks 0 / 1, then the Jr tiles
constexpr int PF_REC = PF_GROUPS * RC_STRIDE;     // doubles: the factor records
// the PF_GROUPS factors of group block `blk`, run by ONE wave (lanes tl = 0..63)
// with its own LDS (tile, rec): the body of preint_factor_kernel and of
// window_factor_kernel's preintegration waves.  Its two __syncthreads are
// reached by every wave of a workgroup (no early exit, dead groups recompute a
// valid factor and store nothing).
__device__ __forceinline__ void preint_factor_body(int blk, double* __restrict__ tile, double* __restrict__ rec, int n,
                                                   const gvx_preint_result* __restrict__ pre,
                                                   const double* __restrict__ pn,
                                                   const int32_t* __restrict__ pn_off,
                                                   const double* __restrict__ params,
                                                   const int32_t* __restrict__ offs, double* __restrict__ res,
                                                   double* __restrict__ jac) {
    static_assert(PF_SLOTS * NS * PF_LD <= PF_TILE, "the tiles fit the pn_ staging");
    const int tl = threadIdx.x & 63;
    const int grp = tl / PF_L, lane = tl % PF_L;
    const int f0 = blk * PF_GROUPS;
    // dead groups (past n, or the partial group) recompute a valid factor and store nothing
    const int fi = min(f0 + min(grp, PF_GROUPS - 1), n - 1);
    const gvx_preint_result* s = pre + fi;
    typedef const __attribute__((address_space(1))) void* gptr;
    typedef __attribute__((address_space(3))) void* lptr;
    // ---- round 1: the records (dwords 0..393: sqrt_info, jacobian block, misc) ----
    // record dword d of factor f comes from struct dword src(d); lane l carries
    // d = 64 j + l of instruction j
    auto src_dword = [&](int d) -> int {
        const int h = d & 1, q = d >> 1;  // double q of the record, half h
        int sd;
        if (q < RC_J6) {  // sqrt_info (r, c), c >= r
            int r = 0;
            while (r < 14 && triu15(r + 1, r + 1) <= q) ++r;
            sd = (int)(offsetof(gvx_preint_result, sqrt_info) / 8) + r * 15 + (r + q - triu15(r, r));
        } else if (q < RC_MISC) {
            const int e = q - RC_J6;
            sd = (int)(offsetof(gvx_preint_result, jacobian) / 8) + (e / 6) * 15 + 9 + e % 6;
        } else if (q == RC_DT) {
            sd = (int)(offsetof(gvx_preint_result, delta_time) / 8);
        } else {
            sd = (int)(offsetof(gvx_preint_result, delta) / 8) + 1 + (q - RC_DP);
        }
        return 2 * sd + h;
    };
    int srcd[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) srcd[j] = src_dword(min(64 * j + tl, 2 * RC_PAR - 1));
#pragma unroll
    for (int f = 0; f < PF_GROUPS; ++f) {
        const uint32_t* sf = reinterpret_cast<const uint32_t*>(pre + min(f0 + f, n - 1));
#pragma unroll
        for (int j = 0; j < 7; ++j)
            if (64 * j + tl < 2 * RC_PAR)
                __builtin_amdgcn_global_load_lds((gptr)(sf + srcd[j]), (lptr)(rec + f * RC_STRIDE + 32 * j), 4, 0, 0);
    }
    const int earth_i = s->variant == GVX_PREINT_EARTH;
    const int m1n = earth_i ? s->m - 1 : 0;
    const int32_t pno = pn_off[fi];
    const int32_t* o = offs + 4 * (int64_t)fi;
    const int o0 = o[0], o1 = o[1], o2 = o[2], o3 = o[3];
    const bool earth = earth_i != 0;
    // ---- round 2: the parameter blocks (record doubles RC_PAR.., 64 dwords) and pn_ ----
    {
        // dword k of [pose0 (14) | mix0 (18) | pose1 (14) | mix1 (18)]
        const int k = tl;
        const int blk = k < 14 ? 0 : (k < 32 ? 1 : (k < 46 ? 2 : 3));
        const int kb = k - (blk == 0 ? 0 : (blk == 1 ? 14 : (blk == 2 ? 32 : 46)));
#pragma unroll
        for (int f = 0; f < PF_GROUPS; ++f) {
            // the offsets of factor f live in group f's lanes
            const int b0 = __shfl(o0, f * PF_L, 64), b1 = __shfl(o1, f * PF_L, 64);
            const int b2 = __shfl(o2, f * PF_L, 64), b3 = __shfl(o3, f * PF_L, 64);
            const int base = blk == 0 ? b0 : (blk == 1 ? b1 : (blk == 2 ? b2 : b3));
            const uint32_t* pp = reinterpret_cast<const uint32_t*>(params + base);
            __builtin_amdgcn_global_load_lds((gptr)(pp + kb), (lptr)(rec + f * RC_STRIDE + RC_PAR), 4, 0, 0);
        }
    }
    // pn_ chunk c0 of this group's factor into LDS half h (instruction j: lane pair
    // (2q, 2q+1) of a group loads sample c0 + PN_PER*j + q, 16 bytes each, to
    // tile + h*1024 + j*128 + group*2*PF_L + q*4 doubles)
    const double* pl = pn + 4 * (int64_t)pno;
    auto pn_chunk = [&](int c0, int h) {
#pragma unroll
        for (int j = 0; j < PN_INS; ++j) {
            const int smp = c0 + PN_PER * j + (lane >> 1);
            if (smp < m1n)
                __builtin_amdgcn_global_load_lds((gptr)(pl + 4 * smp + 2 * (lane & 1)),
                                                 (lptr)(tile + h * PN_INS * 128 + 128 * j), 16, 0, 0);
        }
    };
    pn_chunk(0, 0);
    pn_chunk(PN_CH, 1);
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const double* R = rec + grp * RC_STRIDE;
    const double *ps0 = R + RC_PAR, *m0 = R + RC_PAR + 7, *ps1 = R + RC_PAR + 16, *m1 = R + RC_PAR + 23;
    // Earth: p_cor = sum over pn_ of (pn.second - state0.p) * pn.first
    // (preintegration_earth.cc's loop), lane-parallel: lane l of the group sums
    // the samples k = l mod 16 in order, then a 16-lane butterfly (DPP row_ror)
    // adds the partial sums -- a different association than the reference's
    // sequential loop, within 1e-16 relative (the parity bound is 1e-10)
    double pcs[3] = {0.0, 0.0, 0.0};
    {
        const double p00 = ps0[0], p01 = ps0[1], p02 = ps0[2];
        for (int c0 = 0; __ballot(c0 < m1n); c0 += 2 * PN_CH) {
            if (c0 > 0) {
                pn_chunk(c0, 0);
                pn_chunk(c0 + PN_CH, 1);
                __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const int kn = min(2 * PN_CH, m1n - c0);
            const double* P = tile + 2 * PF_L * grp;
#pragma unroll 4
            for (int k = lane; k < kn; k += PF_L) {
                const int kk = k & (PN_CH - 1);
                const double* e = P + (k >= PN_CH ? PN_INS * 128 : 0) + 128 * (kk / PN_PER) + 4 * (kk % PN_PER);
                const double dt = e[0];
                pcs[0] = pcs[0] + (e[1] - p00) * dt;
                pcs[1] = pcs[1] + (e[2] - p01) * dt;
                pcs[2] = pcs[2] + (e[3] - p02) * dt;
            }
            __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next chunk lands
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            pcs[c] = pcs[c] + dpp_row_ror<8>(pcs[c]);
            pcs[c] = pcs[c] + dpp_row_ror<4>(pcs[c]);
            pcs[c] = pcs[c] + dpp_row_ror<2>(pcs[c]);
            pcs[c] = pcs[c] + dpp_row_ror<1>(pcs[c]);
        }
    }
    // the tile region now holds the Jr tiles
    double* Jr = tile + grp * NS * PF_LD;
    for (int e = lane; e < NS * PF_LD; e += PF_L) Jr[e] = 0.0;
    const dq q0 = dq_make(ps0[6], ps0[3], ps0[4], ps0[5]);
    const dq q1 = dq_make(ps1[6], ps1[3], ps1[4], ps1[5]);
    const double *p0 = ps0, *p1 = ps1, *v0 = m0, *v1 = m1;
    const double *bg0 = m0 + 3, *ba0 = m0 + 6, *bg1 = m1 + 3, *ba1 = m1 + 6;
    // ---- residual and raw Jacobian blocks (uniform over the group) ----
    const double dtt = R[RC_DT];
    const double* J6 = R + RC_J6;
    double dp_dbg[9], dp_dba[9], dv_dbg[9], dv_dba[9], dq_dbg[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            dp_dbg[3 * i + j] = J6[i * 6 + j];
            dp_dba[3 * i + j] = J6[i * 6 + 3 + j];
            dv_dbg[3 * i + j] = J6[(3 + i) * 6 + j];
            dv_dba[3 * i + j] = J6[(3 + i) * 6 + 3 + j];
            dq_dbg[3 * i + j] = J6[(6 + i) * 6 + j];
        }
    double dbg[3], dba[3], t[3], u[3], cp[3], cv[3];
    for (int i = 0; i < 3; ++i) {
        dbg[i] = bg0[i] - R[RC_DBG + i];
        dba[i] = ba0[i] - R[RC_DBA + i];
    }
    mv3(dp_dba, dba, t);
    mv3(dp_dbg, dbg, u);
    for (int i = 0; i < 3; ++i) cp[i] = R[RC_DP + i] + t[i] + u[i];
    mv3(dv_dba, dba, t);
    mv3(dv_dbg, dbg, u);
    for (int i = 0; i < 3; ++i) cv[i] = R[RC_DV + i] + t[i] + u[i];
    mv3(dq_dbg, dbg, t);
    const dq dqd = dq_load(R + RC_DQ);
    const dq cq = dq_mul(dqd, dq_from_rotvec(t));
    const double* g = R + RC_G;
    const double* iewn = R + RC_IEWN;
    const dq q0i = dq_inv(q0);
    double cnb0[9], M[9], N[9];
    dq_rot(q0i, cnb0);
    double r[NS];
    const bool w0 = lane == 0;  // lane 0 of the group writes the uniform blocks
    if (earth) {
        double S[9], S2[9];
        skew(iewn, S);
        double pc[3] = {pcs[0], pcs[1], pcs[2]};
        for (int i = 0; i < 9; ++i) S2[i] = 2.0 * S[i];
        mv3(S2, pc, pc);
        double dp[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]}, vc[3];
        mv3(S2, dp, vc);
        const double dnn[3] = {-iewn[0] * dtt, -iewn[1] * dtt, -iewn[2] * dtt};
        const dq qnn = dq_from_rotvec(dnn);
        double dpn[3], dvn[3];
        for (int i = 0; i < 3; ++i) {
            dpn[i] = p1[i] - p0[i] - v0[i] * dtt - 0.5 * g[i] * dtt * dtt + pc[i];
            dvn[i] = v1[i] - v0[i] - g[i] * dtt + vc[i];
        }
        const dq qb0b1 = dq_mul(dq_mul(dq_inv(q1), qnn), q0);
        mv3(cnb0, dpn, t);
        for (int i = 0; i < 3; ++i) r[i] = t[i] - cp[i];
        mv3(cnb0, dvn, t);
        for (int i = 0; i < 3; ++i) r[3 + i] = t[i] - cv[i];
        const dq e = dq_mul(qb0b1, cq);
        r[6] = 2 * e.x;
        r[7] = 2 * e.y;
        r[8] = 2 * e.z;
        if (jac && w0) {
            // (2 cnb0) S, (-2 cnb0) S and (2 cnb0) S again in the reference: one
            // product scaled by +-2 (exact), the same bits
            mm3(cnb0, S, M);
            for (int i = 0; i < 9; ++i) M[i] = 2.0 * M[i];
            for (int i = 0; i < 9; ++i) N[i] = -cnb0[i] - M[i] * dtt;
            set3(Jr, PF_LD, 0, 0, N);
            mv3(cnb0, dpn, t);
            skew(t, N);
            set3(Jr, PF_LD, 0, 3, N);
            for (int i = 0; i < 9; ++i) N[i] = -M[i];
            set3(Jr, PF_LD, 3, 0, N);
            mv3(cnb0, dvn, t);
            skew(t, N);
            set3(Jr, PF_LD, 3, 3, N);
            qlr_br(qb0b1, cq, N);
            set3(Jr, PF_LD, 6, 3, N);
            // pose1 (columns 16..22)
            set3(Jr, PF_LD, 0, 16, cnb0);
            set3(Jr, PF_LD, 3, 16, M);
            qright_br(dq_mul(qb0b1, cq), N);
            for (int i = 0; i < 9; ++i) N[i] = -N[i];
            set3(Jr, PF_LD, 6, 19, N);
            // mix0 (columns 7..15)
            qleft_br(dq_mul(qb0b1, dqd), M);
            mm3(M, dq_dbg, N);
            set3(Jr, PF_LD, 6, 10, N);
        }
    } else {
        double dp[3], dv[3], rp[3], rv[3];
        for (int i = 0; i < 3; ++i) {
            dp[i] = p1[i] - p0[i] - v0[i] * dtt - 0.5 * g[i] * dtt * dtt;
            dv[i] = v1[i] - v0[i] - g[i] * dtt;
        }
        dq_rotate(q0i, dp, rp);
        dq_rotate(q0i, dv, rv);
        for (int i = 0; i < 3; ++i) {
            r[i] = rp[i] - cp[i];
            r[3 + i] = rv[i] - cv[i];
        }
        const dq e = dq_mul(dq_mul(dq_inv(cq), q0i), q1);
        r[6] = 2 * e.x;
        r[7] = 2 * e.y;
        r[8] = 2 * e.z;
        if (jac && w0) {
            for (int i = 0; i < 9; ++i) N[i] = -cnb0[i];
            set3(Jr, PF_LD, 0, 0, N);
            skew(rp, N);
            set3(Jr, PF_LD, 0, 3, N);
            skew(rv, N);
            set3(Jr, PF_LD, 3, 3, N);
            qlr_br(dq_mul(dq_inv(q1), q0), cq, N);
            for (int i = 0; i < 9; ++i) N[i] = -N[i];
            set3(Jr, PF_LD, 6, 3, N);
            set3(Jr, PF_LD, 0, 16, cnb0);
            qleft_br(e, N);
            set3(Jr, PF_LD, 6, 19, N);
            qleft_br(dq_mul(dq_mul(dq_inv(q1), q0), dqd), M);
            for (int i = 0; i < 9; ++i) M[i] = -M[i];
            mm3(M, dq_dbg, N);
            set3(Jr, PF_LD, 6, 10, N);
        }
    }
    for (int i = 0; i < 3; ++i) {
        r[9 + i] = bg1[i] - bg0[i];
        r[12 + i] = ba1[i] - ba0[i];
    }
    if (jac && w0) {
        // common mix0 / mix1 blocks
        for (int i = 0; i < 9; ++i) N[i] = -cnb0[i] * dtt;
        set3(Jr, PF_LD, 0, 7, N);
        for (int i = 0; i < 9; ++i) N[i] = -dp_dbg[i];
        set3(Jr, PF_LD, 0, 10, N);
        for (int i = 0; i < 9; ++i) N[i] = -dp_dba[i];
        set3(Jr, PF_LD, 0, 13, N);
        for (int i = 0; i < 9; ++i) N[i] = -cnb0[i];
        set3(Jr, PF_LD, 3, 7, N);
        for (int i = 0; i < 9; ++i) N[i] = -dv_dbg[i];
        set3(Jr, PF_LD, 3, 10, N);
        for (int i = 0; i < 9; ++i) N[i] = -dv_dba[i];
        set3(Jr, PF_LD, 3, 13, N);
        for (int i = 0; i < 3; ++i) {
            Jr[(9 + i) * PF_LD + 10 + i] = -1.0;
            Jr[(12 + i) * PF_LD + 13 + i] = -1.0;
            Jr[(9 + i) * PF_LD + 26 + i] = 1.0;
            Jr[(12 + i) * PF_LD + 29 + i] = 1.0;
        }
        set3(Jr, PF_LD, 3, 23, cnb0);
    }
    if (w0)
        for (int i = 0; i < NS; ++i) Jr[i * PF_LD + 32] = r[i];
    // the whitening's A operands (sqrt_info rows / K) of the wave's four factors,
    // from the records' packed upper triangles (sqrt_info is upper triangular)
    const int wl = tl, wr = wl & 15, wk = wl >> 4;
    double SA[PF_GROUPS][4];
#pragma unroll
    for (int f = 0; f < PF_GROUPS; ++f) {
        const double* sq = rec + f * RC_STRIDE + RC_SQ;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int k = 4 * kk + wk;
            SA[f][kk] = (wr < NS && k < NS && k >= wr) ? sq[triu15(wr, k)] : 0.0;
        }
    }
    __syncthreads();
    // ---- whitening: sqrt_info * [Jr | r] on the matrix cores, stored from the
    // accumulators ----
    // Per factor slot f of the wave: three 16-column blocks of the 15 x 33 tile
    // (zero-padded to 16 x 48), each 4 v_mfma_f64_16x16x4 steps over K = 16.
    // Operand layout (16x16x4 f64): A lane l = (row l%16, k l/16), B lane l =
    // (k l/16, col l%16), D lane l = rows l/16 + 4i (i = 0..3) of col l%16
    // (measured: tools/mfma_f64_probe.hip).  The MFMA sums the 15 products in
    // its own order, not the restatement's sequential one; the results stay
    // within 1e-10 of each block's magnitude (tests/test_factor_parity_gpu.py).
    // Each lane writes its four rows of its column straight to the output layout
    // (residual column 32 -> res; Jacobian column c -> block J0 7 | J1 9 | J2 7 |
    // J3 9 of jac), so the tile is not written back and re-read: the block's B
    // reads of all three column blocks are issued before its MFMA chains.
    {
        const int lr = wr, lk = wk;
        const int cb0 = jac ? 0 : 2;  // residual only: the block holding column 32
        const int nf = min(PF_GROUPS, n - f0);
        // the lane's output column in each column block: Jacobian block base,
        // width and column inside it (width 0: column 32, the residual; -1: padding)
        int obase[3], owid[3];
#pragma unroll
        for (int cb = 0; cb < 3; ++cb) {
            const int c = 16 * cb + lr;
            if (c < 7) { obase[cb] = c; owid[cb] = 7; }
            else if (c < 16) { obase[cb] = 105 + (c - 7); owid[cb] = 9; }
            else if (c < 23) { obase[cb] = 240 + (c - 16); owid[cb] = 7; }
            else if (c < 32) { obase[cb] = 345 + (c - 23); owid[cb] = 9; }
            else if (c == 32) { obase[cb] = 0; owid[cb] = 0; }
            else { obase[cb] = 0; owid[cb] = -1; }
        }
        typedef double v4d __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int f = 0; f < PF_GROUPS; ++f) {
            const double* A = SA[f];
            const double* T = tile + f * NS * PF_LD;
            double bv[3][4];
#pragma unroll
            for (int cb = 0; cb < 3; ++cb) {
                const int col = 16 * cb + lr;
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const int k = 4 * kk + lk;
                    bv[cb][kk] = (cb >= cb0 && k < NS && col < PF_LD) ? T[k * PF_LD + col] : 0.0;
                }
            }
            if (f >= nf) continue;  // wave-uniform
            double* rf = res + (int64_t)(f0 + f) * NS;
            double* jf = jac ? jac + (int64_t)(f0 + f) * 480 : nullptr;
#pragma unroll
            for (int cb = 0; cb < 3; ++cb) {
                if (cb < cb0) continue;
                v4d acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[kk], bv[cb][kk], acc, 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int row = lk + 4 * i;
                    if (row >= NS) continue;
                    if (owid[cb] > 0) {
                        if (jf) __builtin_nontemporal_store(acc[i], jf + obase[cb] + row * owid[cb]);
                    } else if (owid[cb] == 0) {
                        __builtin_nontemporal_store(acc[i], rf + row);
                    }
                }
            }
        }
    }
}

__global__ void __launch_bounds__(64) preint_factor_kernel(int n, const gvx_preint_result* __restrict__ pre,
                                                           const double* __restrict__ pn,
                                                           const int32_t* __restrict__ pn_off,
                                                           const double* __restrict__ params,
                                                           const int32_t* __restrict__ offs,
                                                           double* __restrict__ res,
                                                           double* __restrict__ jac) {
    __shared__ double tile[PF_TILE];
    __shared__ double rec[PF_REC];
    preint_factor_body(blockIdx.x, tile, rec, n, pre, pn, pn_off, params, offs, res, jac);
}

// A small window's two factor kinds in ONE launch (a Ceres window: 1,800
// reprojection + 9 preintegration factors): workgroups [0, nbr) are
// reprojection blocks, the rest carry two preintegration waves each, so the
// window costs the longer of the two dependent chains instead of their sum
// (two launches back to back: 29.7 us at r04).  The bodies are the same code
// as the two kernels', so the results are the same bits.
constexpr int WF_LDS = RP_LDS > 2 * (PF_TILE + PF_REC) ? RP_LDS : 2 * (PF_TILE + PF_REC);
__global__ void __launch_bounds__(RP_THREADS) window_factor_kernel(
    int nbr, int n_r, const gvx_reproj_const* __restrict__ cs, const int32_t* __restrict__ roffs,
    double* __restrict__ rres, double* __restrict__ rjac, int n_p, const gvx_preint_result* __restrict__ pre,
    const double* __restrict__ pn, const int32_t* __restrict__ pn_off, const int32_t* __restrict__ poffs,
    double* __restrict__ pres, double* __restrict__ pjac, const double* __restrict__ params) {
    static_assert(RP_THREADS == 128, "two preintegration waves per workgroup");
    __shared__ double lds[WF_LDS];
    if ((int)blockIdx.x < nbr) {
        reproj_body(blockIdx.x, lds, n_r, cs, params, roffs, rres, rjac);
    } else {
        const int w = threadIdx.x >> 6;
        double* tile = lds + w * (PF_TILE + PF_REC);
        preint_factor_body(2 * ((int)blockIdx.x - nbr) + w, tile, tile + PF_TILE, n_p, pre, pn, pn_off, params, poffs,
                           pres, pjac);
    }
}

}  // namespace

hipError_t launch_window_factors(gvx_ctx* c, int n_r, const gvx_reproj_const* cs, const int32_t* roffs, double* rres,
                                 double* rjac, int n_p, const gvx_preint_result* pre, const double* pn,
                                 const int32_t* pn_off, const int32_t* poffs, double* pres, double* pjac,
                                 const double* params) {
    const int nbr = (n_r + RP_THREADS - 1) / RP_THREADS;
    const int nbp = ((n_p + PF_GROUPS - 1) / PF_GROUPS + 1) / 2;
    if (nbr + nbp == 0) return hipSuccess;
    return launch_timed(c, "factor_window", window_factor_kernel, dim3(nbr + nbp), dim3(RP_THREADS), 0, nbr, n_r, cs,
                        roffs, rres, rjac, n_p, pre, pn, pn_off, poffs, pres, pjac, params);
}

// the fused launch takes windows whose blocks fill at most this many workgroups
// per CU (the batched launches beyond it: the two kernels are tuned apart)
int window_factor_blocks(int n_r, int n_p) {
    return (n_r + RP_THREADS - 1) / RP_THREADS + ((n_p + PF_GROUPS - 1) / PF_GROUPS + 1) / 2;
}

hipError_t launch_reproj(gvx_ctx* c, int n, const gvx_reproj_const* cs, const double* params,
                         const int32_t* offs, double* res, double* jac) {
    if (n <= 0) return hipSuccess;
    return launch_timed(c, "reproj", reproj_kernel, dim3((n + RP_THREADS - 1) / RP_THREADS), dim3(RP_THREADS), 0, n,
                        cs, params, offs, res, jac);
}

hipError_t launch_preint_factor(gvx_ctx* c, int n, const gvx_preint_result* pre, const double* pn,
                                const int32_t* pn_off, const double* params, const int32_t* offs,
                                double* res, double* jac) {
    if (n <= 0) return hipSuccess;
    return launch_timed(c, "preint_factor", preint_factor_kernel, dim3((n + PF_GROUPS - 1) / PF_GROUPS), dim3(64), 0,
                        n, pre, pn, pn_off, params, offs, res, jac);
}

hipError_t launch_sqrt_info(gvx_ctx* c, int n, gvx_preint_result* pre) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(sqrt_info_kernel, dim3((n + SQ_SEG - 1) / SQ_SEG), dim3(64), 0, c->stream, n, pre);
    return hipGetLastError();
}

}  // namespace gvx
