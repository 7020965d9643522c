// preint.hip -- batched IMU preintegration for gfx950 (fp64).
//
// Replaces Preintegration::createPreintegration + addNewImu for k = 1..m-1
// (/root/reference/ic_gvins/ic_gvins/ic_gvins.cc:946-953) for both reachable
// variants: PreintegrationNormal (preintegration_normal.cc:183-232 with
// preintegration_base.cc:39-70) and PreintegrationEarth
// (preintegration_earth.cc:205-303).
//
// One 64-lane wavefront per segment; the scan over IMU samples is sequential.
// Per step every lane evaluates the (uniform) state update, then the 15x15
// products J <- Phi J and P <- Phi P Phi^T + Qk are spread over the lanes
// (entries e = lane + 64 r).  Phi, G and the noise are structurally sparse; the
// sparse sums visit the non-zero terms in ascending k like the dense products
// of the reference (adding an exact 0*x never changes a non-zero sum), so the
// GPU J/P match the sequential CPU restatement up to the fp64 sin/cos of the
// rotation-vector exponentials and the fused multiply-adds of phi_mv.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdlib>

#include "dmath.h"
#include "gvx_internal.h"

namespace gvx {

namespace {

constexpr int NS = 15;

// q / |q| through one reciprocal square root (v_rsq_f64 and two fused Newton
// steps) instead of a square root and four divisions: within an ulp or two of
// Eigen's normalized(), and a shorter dependent chain for the quaternion
// recursions (their contract is 1e-10 relative)
__device__ __forceinline__ dq dq_renorm(dq q) {
    const double n2 = dq_sqnorm(q);
    if (n2 > 0) {
        double y = __builtin_amdgcn_rsq(n2);
        double e = __builtin_fma(-n2 * y, y, 1.0);
        y = __builtin_fma(0.5 * y, e, y);
        e = __builtin_fma(-n2 * y, y, 1.0);
        y = __builtin_fma(0.5 * y, e, y);
        q.x *= y;
        q.y *= y;
        q.z *= y;
        q.w *= y;
    }
    return q;
}

// Every kernel below is one wavefront per workgroup: its LDS traffic is in order
// within the wave, so a step's hand-over through LDS needs a compiler fence, not
// s_barrier and the lgkmcnt(0) drain in front of it.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct Imu {
    double dt, dth[3], dv[3], time;
};

// rotvec2quaternion (Eigen AngleAxis: (cos(a/2), sin(a/2) r/|r|)) for the
// small angles of one IMU sample and of the Earth rotation over a segment:
// with y = |r|^2 / 4, cos(a/2) and sin(a/2)/|r| are even series in |r|, so no
// square root, division or sin / cos call is needed.  Below y = 2.5e-3 (an
// angle of 0.1 rad) the series are cut after the y^5 / y^4 terms, whose
// remainders are < 1e-20 relative; larger angles take dmath's exact form.
// Differs from it by rounding only (1e-16), inside the 1e-10 contract; a
// preintegration step computes four of these (r05: ~40 % of the pre pass).
__device__ __attribute__((noinline)) dq dq_from_rotvec_large(double r0, double r1, double r2) {
    const double r[3] = {r0, r1, r2};
    return dq_from_rotvec(r);
}
__device__ __forceinline__ dq dq_from_rotvec_small(const double* r) {
    const double n2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
    const double y = 0.25 * n2;
    if (y > 2.5e-3) return dq_from_rotvec_large(r[0], r[1], r[2]);  // out of line: rare
    // cos x = 1 - y/2 + y^2/24 - y^3/720 + y^4/40320 - y^5/3628800 (x^2 = y)
    double c = __builtin_fma(y, -1.0 / 3628800.0, 1.0 / 40320.0);
    c = __builtin_fma(y, c, -1.0 / 720.0);
    c = __builtin_fma(y, c, 1.0 / 24.0);
    c = __builtin_fma(y, c, -0.5);
    c = __builtin_fma(y, c, 1.0);
    // sin x / (2 x) = (1 - y/6 + y^2/120 - y^3/5040 + y^4/362880) / 2
    double t = __builtin_fma(y, 1.0 / 362880.0, -1.0 / 5040.0);
    t = __builtin_fma(y, t, 1.0 / 120.0);
    t = __builtin_fma(y, t, -1.0 / 6.0);
    t = __builtin_fma(y, t, 1.0);
    t *= 0.5;
    return dq_make(c, t * r[0], t * r[1], t * r[2]);
}

__device__ __forceinline__ Imu load_imu(const gvx_imu* p, const double* bg, const double* ba) {
    // PreintegrationBase::compensationBias (preintegration_base.cc:86-92)
    Imu r;
    r.time = p->time;
    r.dt = p->dt;
    for (int i = 0; i < 3; ++i) {
        r.dth[i] = p->dtheta[i] - p->dt * bg[i];
        r.dv[i] = p->dvel[i] - p->dt * ba[i];
    }
    return r;
}

// Quantities of step k that depend only on the IMU samples, the (constant)
// biases, iewn and the running delta_time -- not on the recursion.  They
// carry all the transcendental work (rotvec2quaternion) and are computed for
// CH steps at once, one step per lane, before the sequential part.
struct StepPre {
    double dt, time, dtime;    // dt, sample time, delta_time after this step
    double dvfb[3];            // two-sample sculling (preintegration_base.cc:47-48)
    double dv[3], dth[3];      // bias-compensated dvel / dtheta (Phi's C and M blocks)
    double qd[4];              // rotvec2quaternion(dtheta + coning)
    double qnn[4];             // Earth: rotvec2quaternion(-iewn dt)
    double qa[4], qb[4];       // Earth: q0^-1 q(-(dtime - dt/2) iewn) q0, q0^-1 q(-dtime iewn) q0
};
constexpr int PRE_DW = sizeof(StepPre) / 8;

// Sparse Phi (updateJacobianAndCovariance: preintegration_base.cc:94-125,
// preintegration_earth.cc:266-303) applied to one column vector; terms in
// ascending k like the dense product, each multiply-add fused (one rounding
// instead of Eigen's two: 1e-16 relative per step, inside the 1e-10 contract;
// 0.418 -> 0.390 ms per configs[3] launch, profiles/r04_v12/cov).
struct Phi {
    double dt, f;        // Phi(0:3, 3:6) = dt I ; Phi(9:15, 9:15) = (1 - dt/T) I
    double C[9];         // Phi(3:6, 6:9) = cbb0 * skew(dvel)
    double D[9];         // Phi(3:6, 12:15) = cbb0 * dt
    double M[9];         // Phi(6:9, 6:9) = I - skew(dtheta); Phi(6:9, 9:12) = -dt I
};

// Phi with its (6:9, 6:9) block as dtheta (the covariance pass's record prefix:
// 24 doubles a step instead of 29 in registers and 12 b128 reads instead of 15)
struct PhiT {
    double dt, f;
    double C[9], D[9];
    double th[3], pad;
};
// phi_mv with M = I - skew(th) formed in the products: its entries are exact
// (0 - (-x) = x, 1 - 0 = 1), 1 * v6 is v6 and fma(1, v7, s) rounds like
// s + v7, so the result has the same bits as phi_mv's
__device__ __forceinline__ void phi_mv_t(const PhiT& f, const double* v, double* y) {
#pragma unroll
    for (int i = 0; i < 3; ++i) y[i] = __builtin_fma(f.dt, v[3 + i], v[i]);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        double s = v[3 + a];
        s = __builtin_fma(f.C[3 * a], v[6], s);
        s = __builtin_fma(f.C[3 * a + 1], v[7], s);
        s = __builtin_fma(f.C[3 * a + 2], v[8], s);
        s = __builtin_fma(f.D[3 * a], v[12], s);
        s = __builtin_fma(f.D[3 * a + 1], v[13], s);
        s = __builtin_fma(f.D[3 * a + 2], v[14], s);
        y[3 + a] = s;
    }
    // rows of I - skew(th): (1, th2, -th1), (-th2, 1, th0), (th1, -th0, 1)
    double s = v[6];
    s = __builtin_fma(f.th[2], v[7], s);
    s = __builtin_fma(-f.th[1], v[8], s);
    y[6] = __builtin_fma(-f.dt, v[9], s);
    s = -f.th[2] * v[6];
    s = s + v[7];
    s = __builtin_fma(f.th[0], v[8], s);
    y[7] = __builtin_fma(-f.dt, v[10], s);
    s = f.th[1] * v[6];
    s = __builtin_fma(-f.th[0], v[7], s);
    s = s + v[8];
    y[8] = __builtin_fma(-f.dt, v[11], s);
#pragma unroll
    for (int i = 9; i < NS; ++i) y[i] = f.f * v[i];
}

__device__ __forceinline__ void phi_mv(const Phi& f, const double* v, double* y) {
#pragma unroll
    for (int i = 0; i < 3; ++i) y[i] = __builtin_fma(f.dt, v[3 + i], v[i]);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        double s = v[3 + a];
        s = __builtin_fma(f.C[3 * a], v[6], s);
        s = __builtin_fma(f.C[3 * a + 1], v[7], s);
        s = __builtin_fma(f.C[3 * a + 2], v[8], s);
        s = __builtin_fma(f.D[3 * a], v[12], s);
        s = __builtin_fma(f.D[3 * a + 1], v[13], s);
        s = __builtin_fma(f.D[3 * a + 2], v[14], s);
        y[3 + a] = s;
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        double s = f.M[3 * a] * v[6];
        s = __builtin_fma(f.M[3 * a + 1], v[7], s);
        s = __builtin_fma(f.M[3 * a + 2], v[8], s);
        s = __builtin_fma(-f.dt, v[9 + a], s);
        y[6 + a] = s;
    }
#pragma unroll
    for (int i = 9; i < NS; ++i) y[i] = f.f * v[i];
}

// P'(:,c) = Phi K + a W phi_c for rows 3..14 (rows 0..2 have no Q term): the
// W(3:6,3:6) block times phi_c(3:6) and the constant diagonal of W from row 6 on
// (wg, nbg, nba), multiply-adds fused.  Shared by every covariance kernel so
// their outputs stay the same bits.
__device__ __forceinline__ void q_terms(double a, const double* W, double wg, double nbg, double nba,
                                        const double* ph, const double* y, double* P) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        double u = W[3 * i] * ph[3];
        u = __builtin_fma(W[3 * i + 1], ph[4], u);
        u = __builtin_fma(W[3 * i + 2], ph[5], u);
        P[3 + i] = __builtin_fma(a, u, y[3 + i]);
    }
    const double ag = a * wg, abg = a * nbg, aba = a * nba;
#pragma unroll
    for (int i = 6; i < 15; ++i) P[i] = __builtin_fma(i < 9 ? ag : (i < 12 ? abg : aba), ph[i], y[i]);
}

constexpr int GL = 16;                  // lanes per segment: lane c owns column c of J and row c of P
constexpr int SPW = 64 / GL;            // segments per (one-wave) workgroup
constexpr int CH = GL;                  // steps per precompute chunk (one per lane)
constexpr int MS = NS * NS;

// One wavefront = 4 segments x 16 lanes.  Per IMU step:
//   * the state recursion (cheap once the StepPre terms exist) runs redundantly
//     on the 16 lanes of a segment, so Phi's blocks are in every lane's registers;
//   * J <- Phi J: lane c updates column c (sparse mat-vec, 45 MAC);
//   * P <- Phi P Phi^T + Qk, Qk = a (Phi W + W Phi^T), a = dt/2, W = gt N gt^T
//     (block diagonal): lane c writes G(:,c) = Phi P(:,c) to LDS and reads row
//     c back; with P symmetric, P Phi^T = G^T, so
//     P'(:,c) = Phi (G(c,:)^T + a W(:,c)) + a W Phi(c,:)^T.
// Sums are reassociated against the dense Eigen products (relative 1e-16 per
// step); the parity bound is 1e-10 of each block's magnitude (tests/test_ba_gpu.py).
__global__ void __launch_bounds__(64) preint_kernel(int variant, gvx_imu_params prm, int n_seg,
                                                    const gvx_imu* __restrict__ imu,
                                                    const int32_t* __restrict__ seg_off,
                                                    const gvx_state* __restrict__ state0,
                                                    const double* __restrict__ iewn_in,
                                                    gvx_preint_result* __restrict__ out,
                                                    double* __restrict__ pn) {
    __shared__ double sPre[SPW][CH][PRE_DW];
    __shared__ double sG[SPW][MS];
    const int lane = threadIdx.x;
    const int grp = lane / GL, c = lane % GL;
    const int seg = blockIdx.x * SPW + grp;
    const bool live = seg < n_seg;
    const int b0 = live ? seg_off[seg] : 0;
    const int m = live ? seg_off[seg + 1] - b0 : 0;
    // wave-uniform trip count over the 4 segments (ragged m)
    int mmax = m;
#pragma unroll
    for (int o = GL; o < 64; o <<= 1) mmax = max(mmax, __shfl_xor(mmax, o));
    const gvx_imu* im = imu + b0;
    double* pns = (pn && live) ? pn + (size_t)(b0 - seg) * 4 : nullptr;
    const bool earth = variant == GVX_PREINT_EARTH;

    // ---- constructor: resetState(state, NUM_STATE) + setNoiseMatrix ----
    gvx_state cur = live ? state0[seg] : gvx_state{};
    double dp[3] = {0, 0, 0}, dv[3] = {0, 0, 0};
    dq dqt = dq_make(1, 0, 0, 0);
    double bg[3], ba[3];
    for (int i = 0; i < 3; ++i) {
        bg[i] = cur.bg[i];
        ba[i] = cur.ba[i];
    }
    const dq q0 = dq_load(cur.q);
    const dq q0i = dq_inv(q0);
    double iewn[3] = {0, 0, 0};
    if (earth && live)
        for (int i = 0; i < 3; ++i) iewn[i] = iewn_in[3 * seg + i];
    const double g3[3] = {0, 0, prm.gravity};
    const double ngyr = prm.gyr_arw * prm.gyr_arw, nacc = prm.acc_vrw * prm.acc_vrw;
    const double nbg = 2 * prm.gyr_bias_std * prm.gyr_bias_std / prm.corr_time;
    const double nba = 2 * prm.acc_bias_std * prm.acc_bias_std / prm.corr_time;
    const double g60 = earth ? -1.0 : 1.0;
    const double wg = (g60 * ngyr) * g60;
    // W's constant diagonal from row 6 on: (g60 N_g g60, N_bg, N_ba)
    auto wd = [&](int i) { return i < 9 ? wg : (i < 12 ? nbg : nba); };
    double Jc[NS], Pc[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        Jc[i] = i == c ? 1.0 : 0.0;
        Pc[i] = 0.0;
    }
    double delta_time = 0.0;
    double* pre_base = &sPre[grp][0][0];

    for (int kc = 1; kc < mmax; kc += CH) {
        // ---- precompute StepPre for steps kc .. kc+CH-1, one per lane ----
        {
            const int k = kc + c;
            StepPre sp;
            if (k < m) {
                const Imu pr = load_imu(im + k - 1, bg, ba);
                const Imu ic = load_imu(im + k, bg, ba);
                double dtime = delta_time;
                for (int i = kc; i <= k; ++i) dtime += im[i].dt;  // sequential, as delta_time_ += dt
                sp.dt = ic.dt;
                sp.time = ic.time;
                sp.dtime = dtime;
                double c1[3], c2[3], c3[3], dth[3];
                cross3(ic.dth, ic.dv, c1);
                cross3(pr.dth, ic.dv, c2);
                cross3(pr.dv, ic.dth, c3);
                for (int i = 0; i < 3; ++i) sp.dvfb[i] = ic.dv[i] + 0.5 * c1[i] + 1.0 / 12.0 * (c2[i] + c3[i]);
                cross3(pr.dth, ic.dth, c1);
                for (int i = 0; i < 3; ++i) {
                    dth[i] = ic.dth[i] + 1.0 / 12.0 * c1[i];
                    sp.dv[i] = ic.dv[i];
                    sp.dth[i] = ic.dth[i];
                }
                dq_store(dq_from_rotvec_small(dth), sp.qd);
                if (earth) {
                    const double dt = ic.dt;
                    const double dnn[3] = {-iewn[0] * dt, -iewn[1] * dt, -iewn[2] * dt};
                    dq_store(dq_from_rotvec_small(dnn), sp.qnn);
                    const double sc = -(dtime - 0.5 * dt);
                    const double dnn2[3] = {sc * iewn[0], sc * iewn[1], sc * iewn[2]};
                    dq_store(dq_mul(dq_mul(q0i, dq_from_rotvec_small(dnn2)), q0), sp.qa);
                    const double dnn3[3] = {-iewn[0] * dtime, -iewn[1] * dtime, -iewn[2] * dtime};
                    dq_store(dq_mul(dq_mul(q0i, dq_from_rotvec_small(dnn3)), q0), sp.qb);
                }
                const double* w = reinterpret_cast<const double*>(&sp);
                double* dst = pre_base + c * PRE_DW;
                for (int i = 0; i < PRE_DW; ++i) dst[i] = w[i];
            }
        }
        wave_lds_sync();
        const int kend = min(kc + CH, mmax);
        for (int k = kc; k < kend; ++k) {
            const bool act = k < m;
            Phi f;
            double Wv[9];
            if (act) {
                const StepPre& sp = *reinterpret_cast<const StepPre*>(pre_base + (k - kc) * PRE_DW);
                const double dt = sp.dt;
                delta_time = sp.dtime;
                const dq qd = dq_load(sp.qd);
                double R[9], dvel[3], cbb0[9];
                if (!earth) {
                    // PreintegrationNormal::integrationProcess (preintegration_normal.cc:183-214)
                    dq_rot(dq_load(cur.q), R);
                    mv3(R, sp.dvfb, dvel);
                    for (int i = 0; i < 3; ++i) dvel[i] = dvel[i] + g3[i] * dt;
                    for (int i = 0; i < 3; ++i) cur.p[i] += dt * cur.v[i] + 0.5 * dt * dvel[i];
                    for (int i = 0; i < 3; ++i) cur.v[i] += dvel[i];
                    dq_store(dq_renorm(dq_mul(dq_load(cur.q), qd)), cur.q);
                    dq_rot(dqt, R);
                    mv3(R, sp.dvfb, dvel);
                    for (int i = 0; i < 3; ++i) dp[i] += dt * dv[i] + 0.5 * dt * dvel[i];
                    for (int i = 0; i < 3; ++i) dv[i] += dvel[i];
                    dqt = dq_renorm(dq_mul(dqt, qd));
                    dq_rot(dqt, R);
                    for (int i = 0; i < 9; ++i) cbb0[i] = -R[i];
                } else {
                    // PreintegrationEarth::integrationProcess (preintegration_earth.cc:205-260)
                    double cc[3], dvcg[3], T[9], M1[9];
                    cross3(iewn, cur.v, cc);
                    for (int i = 0; i < 3; ++i) dvcg[i] = (g3[i] - 2.0 * cc[i]) * dt;
                    dq_rot(dq_load(sp.qnn), T);
                    for (int i = 0; i < 9; ++i) M1[i] = 0.5 * (((i % 4) == 0 ? 1.0 : 0.0) + T[i]);
                    dq_rot(dq_load(cur.q), R);
                    mm3(M1, R, T);
                    mv3(T, sp.dvfb, dvel);
                    for (int i = 0; i < 3; ++i) dvel[i] = dvel[i] + dvcg[i];
                    for (int i = 0; i < 3; ++i) cur.p[i] += dt * cur.v[i] + 0.5 * dt * dvel[i];
                    for (int i = 0; i < 3; ++i) cur.v[i] += dvel[i];
                    if (pns && c == 0) {
                        pns[4 * (k - 1)] = dt;
                        pns[4 * (k - 1) + 1] = cur.p[0];
                        pns[4 * (k - 1) + 2] = cur.p[1];
                        pns[4 * (k - 1) + 3] = cur.p[2];
                    }
                    dq_store(dq_renorm(dq_mul(dq_mul(dq_load(sp.qnn), dq_load(cur.q)), qd)), cur.q);
                    dq_rot(dq_mul(dq_load(sp.qa), dqt), R);
                    mv3(R, sp.dvfb, dvel);
                    for (int i = 0; i < 3; ++i) dp[i] += dt * dv[i] + 0.5 * dt * dvel[i];
                    for (int i = 0; i < 3; ++i) dv[i] += dvel[i];
                    dqt = dq_renorm(dq_mul(dqt, qd));
                    dq_rot(dq_mul(dq_load(sp.qb), dqt), R);
                    for (int i = 0; i < 9; ++i) cbb0[i] = -R[i];
                }
                cur.time = sp.time;
                // gt(3:6, 3:6) = R (Normal) or cbb0 (Earth); W(3:6, 3:6) = gR N_v gR^T
                const double sg = earth ? 1.0 : -1.0;  // gR = sg * cbb0
                double gR[9];
                for (int i = 0; i < 9; ++i) gR[i] = sg * cbb0[i];
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b) {
                        double g = (gR[3 * a] * nacc) * gR[3 * b];
                        g = g + (gR[3 * a + 1] * nacc) * gR[3 * b + 1];
                        g = g + (gR[3 * a + 2] * nacc) * gR[3 * b + 2];
                        Wv[3 * a + b] = g;
                    }
                double S[9];
                skew(sp.dv, S);
                mm3(cbb0, S, f.C);
                for (int i = 0; i < 9; ++i) f.D[i] = cbb0[i] * dt;
                skew(sp.dth, S);
                for (int i = 0; i < 9; ++i) f.M[i] = ((i % 4) == 0 ? 1.0 : 0.0) - S[i];
                f.dt = dt;
                f.f = 1 - dt / prm.corr_time;

                // G(:,c) = Phi P(:,c) to LDS; J <- Phi J
                double y[NS];
                phi_mv(f, Pc, y);
                if (c < NS) {
#pragma unroll
                    for (int i = 0; i < NS; ++i) sG[grp][c * NS + i] = y[i];
                }
                phi_mv(f, Jc, y);
#pragma unroll
                for (int i = 0; i < NS; ++i) Jc[i] = y[i];
            }
            wave_lds_sync();
            if (act) {
                const double a = 0.5 * f.dt;
                const int cl = c < NS ? c : 0;
                // K(:,c) = G(c,:)^T + a W(:,c)   (P symmetric: P Phi^T = (Phi P)^T)
                double K[NS];
#pragma unroll
                for (int i = 0; i < NS; ++i) K[i] = sG[grp][i * NS + cl];
                if (c >= 3 && c < 6) {
                    K[3] = K[3] + a * Wv[c - 3];
                    K[4] = K[4] + a * Wv[3 + c - 3];
                    K[5] = K[5] + a * Wv[6 + c - 3];
                }
#pragma unroll
                for (int i = 6; i < NS; ++i)
                    if (i == c) K[i] = K[i] + a * wd(i);
                // phi_c = row c of Phi (lane-dependent selects)
                const int r3 = c - 3, r6 = c - 6;
                double ph[NS];
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    ph[3 + b] = (c == b) ? f.dt : (c == 3 + b ? 1.0 : 0.0);
                    const double cr = r3 == 0 ? f.C[b] : (r3 == 1 ? f.C[3 + b] : f.C[6 + b]);
                    const double mr = r6 == 0 ? f.M[b] : (r6 == 1 ? f.M[3 + b] : f.M[6 + b]);
                    const double dr = r3 == 0 ? f.D[b] : (r3 == 1 ? f.D[3 + b] : f.D[6 + b]);
                    ph[6 + b] = (r3 >= 0 && r3 < 3) ? cr : ((r6 >= 0 && r6 < 3) ? mr : 0.0);
                    ph[9 + b] = (c == 6 + b) ? -f.dt : (c == 9 + b ? f.f : 0.0);
                    ph[12 + b] = (r3 >= 0 && r3 < 3) ? dr : (c == 12 + b ? f.f : 0.0);
                }
                // P'(:,c) = Phi K(:,c) + a W phi_c
                double y[NS];
                phi_mv(f, K, y);
#pragma unroll
                for (int i = 0; i < 3; ++i) Pc[i] = y[i];
                q_terms(a, Wv, wg, nbg, nba, ph, y, Pc);
            }
            wave_lds_sync();
        }
    }

    // ---- outputs ----
    if (!live) return;
    gvx_preint_result* o = out + seg;
    if (c < NS) {
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            o->jacobian[i * NS + c] = Jc[i];
            o->covariance[c * NS + i] = Pc[i];
        }
    }
    if (c == 0) {
        o->variant = variant;
        o->m = m;
        o->delta_time = delta_time;
        o->start_time = im[0].time;
        o->end_time = m > 1 ? im[m - 1].time : im[0].time;
        o->current = cur;
        gvx_state d;
        d.time = 0;
        for (int i = 0; i < 3; ++i) {
            d.p[i] = dp[i];
            d.v[i] = dv[i];
            d.bg[i] = bg[i];
            d.ba[i] = ba[i];
            o->gravity[i] = g3[i];
            o->iewn[i] = iewn[i];
        }
        dq_store(dqt, d.q);
        o->delta = d;
        dq_store(q0, o->q0);
    }
}

// ------------------------------------------------ two-launch preintegration
// preint_kernel's sequential part runs on every lane of a wave that serves 4
// segments: the wave's issue time per step is the same whether it advances 4
// segments or 64, and 5,247 segments give 1.3 k such waves for 1,024 SIMDs.
// Of that part only the two quaternion chains (cur.q and the delta rotation
// dqt) and the velocity / position sums are truly sequential; the rotation
// matrices and rotated increments of a step follow from the chain values, and
// the chains themselves are products of per-step quaternions.  So:
//   preint_pre_kernel    one lane per STEP (a workgroup per segment): the
//                        StepPre terms -- every transcendental of the step --
//                        and the two chains as wave-wide prefix products;
//   preint_cov16_kernel  16 lanes per segment: the step records (rotated terms,
//                        Phi, W) formed 8 steps at a time, one step per lane,
//                        then the velocity / position sums, J <- Phi J and
//                        P <- Phi P Phi^T + Qk per step, sqrt_info at the end.
// Every other value is formed by the same operations in the same order as in
// preint_kernel (tests/test_ba_gpu.py).
// What the covariance pass needs of step k (scratch, one record per IMU step,
// written by preint_pre_kernel): the bias-compensated sample, the rotation whose
// negated matrix is cbb0 and the rotated velocity / delta-velocity increments
// (the reference's integrationProcess terms, preintegration_earth.cc:205-260,
// preintegration_normal.cc:183-214).
struct CovIn {
    double dt, sdth[3], sdv[3];
    double qc[4];  // cbb0 = -R(qc): qc = dqt_k (Normal), q0^-1 q(-dtime iewn) q0 dqt_k (Earth)
    double a[3], b[3];
    double pad;
};
constexpr int COVIN_DW = sizeof(CovIn) / 8;  // 18 (144 B)
static_assert(sizeof(CovIn) % 16 == 0, "16-B records (LDS-DMA pieces)");
constexpr size_t STEP_SCRATCH = sizeof(CovIn);  // per IMU sample

// A quaternion through one DPP lane move (both dwords of each double); lanes
// the move does not write (rows off ROWS, or a row shift's first lanes) take
// the identity
template <int CTRL, int ROWS>
__device__ __forceinline__ dq dq_dpp(dq v) {
    const auto mv = [](double x, double o) -> double {
        const int lo = __builtin_amdgcn_update_dpp(__double2loint(o), __double2loint(x), CTRL, ROWS, 0xf, false);
        const int hi = __builtin_amdgcn_update_dpp(__double2hiint(o), __double2hiint(x), CTRL, ROWS, 0xf, false);
        return __hiloint2double(hi, lo);
    };
    return dq{mv(v.x, 0.0), mv(v.y, 0.0), mv(v.z, 0.0), mv(v.w, 1.0)};
}
// Inclusive prefix products of one quaternion per lane over the wave, in lane
// order (Hillis-Steele: row shifts by 1, 2, 4, 8 inside each 16-lane row, then
// the row totals by row_bcast:15 and row_bcast:31).  RIGHT: P_i = x_0 x_1 .. x_i
// (later factors on the right); else P_i = x_i .. x_1 x_0.
template <bool RIGHT>
__device__ __forceinline__ dq wave_prefix_product(dq p) {
    const auto comb = [](dq lower, dq self) { return RIGHT ? dq_mul(lower, self) : dq_mul(self, lower); };
    p = comb(dq_dpp<0x111, 0xf>(p), p);
    p = comb(dq_dpp<0x112, 0xf>(p), p);
    p = comb(dq_dpp<0x114, 0xf>(p), p);
    p = comb(dq_dpp<0x118, 0xf>(p), p);
    p = comb(dq_dpp<0x142, 0xa>(p), p);
    p = comb(dq_dpp<0x143, 0xc>(p), p);
    return p;
}
// lane i - 1's quaternion (DPP wave_shr:1); lane 0 takes `first`
// inclusive wave prefix sum of a double (lanes past the data carry 0), the
// same DPP ladder as wave_prefix_product
template <int CTRL, int ROWS>
__device__ __forceinline__ double d_dpp(double x) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, ROWS, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, ROWS, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_prefix_sum(double x) {
    x = d_dpp<0x111, 0xf>(x) + x;
    x = d_dpp<0x112, 0xf>(x) + x;
    x = d_dpp<0x114, 0xf>(x) + x;
    x = d_dpp<0x118, 0xf>(x) + x;
    x = d_dpp<0x142, 0xa>(x) + x;
    x = d_dpp<0x143, 0xc>(x) + x;
    return x;
}

__device__ __forceinline__ dq dq_wave_shr1(dq v, dq first) {
    const auto mv = [](double x, double o) -> double {
        const int lo = __builtin_amdgcn_update_dpp(__double2loint(o), __double2loint(x), 0x138, 0xf, 0xf, false);
        const int hi = __builtin_amdgcn_update_dpp(__double2hiint(o), __double2hiint(x), 0x138, 0xf, 0xf, false);
        return __hiloint2double(hi, lo);
    };
    return dq{mv(v.x, first.x), mv(v.y, first.y), mv(v.z, first.z), mv(v.w, first.w)};
}
__device__ __forceinline__ double d_readlane(double x, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                            __builtin_amdgcn_readlane(__double2loint(x), l));
}
__device__ __forceinline__ dq dq_readlane(dq v, int l) {
    return dq{d_readlane(v.x, l), d_readlane(v.y, l), d_readlane(v.z, l), d_readlane(v.w, l)};
}

// The per-step terms and the quaternion chains of one segment (one wave, lane =
// step).  The chains are products: the reference's
//     cur.q_k = normalize(qnn_k * cur.q_k-1 * qd_k)   (Normal: cur.q_k-1 * qd_k)
//     dqt_k   = normalize(dqt_k-1 * qd_k)
// normalise a product that is a unit quaternion up to rounding at every step,
// so cur.q_k = normalize(L_k q0 R_k) and dqt_k = normalize(R_k) with the prefix
// products R_k = qd_1 .. qd_k and L_k = qnn_k .. qnn_1 -- each a wave-wide scan
// of the chunk's 64 steps (6 DPP stages) times the previous chunks' carry,
// instead of a 99-step dependent chain on one lane per segment (the r04 chain
// pass: 50 us per configs[3] batch, 1,200 cycles a step).  The two forms agree
// to rounding (1e-15 relative on configs[3]; tests/test_ba_gpu.py holds the
// whole integration to the oracle at 1e-10).
template <bool EARTH>
__global__ void __launch_bounds__(64, EARTH ? 4 : 6) preint_pre_kernel(int seg0, const gvx_imu* __restrict__ imu,
                                                        const int32_t* __restrict__ seg_off,
                                                        const gvx_state* __restrict__ state0,
                                                        const double* __restrict__ iewn_in,
                                                        CovIn* __restrict__ cin, gvx_imu_params prm,
                                                        gvx_preint_result* __restrict__ out) {
    const int seg = seg0 + blockIdx.x;
    const int lane = threadIdx.x;
    const int b0 = seg_off[seg];
    const int m = seg_off[seg + 1] - b0;
    const gvx_imu* im = imu + b0;
    CovIn* cs = cin + (b0 - seg);
    const gvx_state& s0 = state0[seg];
    double bg[3], ba[3], iewn[3] = {0, 0, 0};
    for (int i = 0; i < 3; ++i) {
        bg[i] = s0.bg[i];
        ba[i] = s0.ba[i];
    }
    const dq q0 = dq_load(s0.q);
    const dq q0i = dq_inv(q0);
    if (EARTH)
        for (int i = 0; i < 3; ++i) iewn[i] = iewn_in[3 * seg + i];
    gvx_preint_result* o = out + seg;
    dq Rc = dq_make(1, 0, 0, 0), Lc = dq_make(1, 0, 0, 0);  // the previous chunks' products
    dq qlast = q0;  // the attitude after the previous chunk's last step (Rc: its delta)
    double base = 0.0;  // delta_time before the chunk
    for (int kc = 1; kc < m; kc += 64) {
        const int k = kc + lane;
        const bool live = k < m;
        // delta_time_ += dt: a wave prefix sum over the chunk's samples on top
        // of the previous chunks' total (summation order differs from the
        // sequential sum by rounding: 1e-16 relative, inside the 1e-10 contract;
        // the lane-by-lane running sum was 64 dependent cross-lane reads a chunk)
        const double mydt = live ? im[k].dt : 0.0;
        const double dtime = base + wave_prefix_sum(mydt);
        base = d_readlane(dtime, 63);
        dq qd = dq_make(1, 0, 0, 0), qnn = dq_make(1, 0, 0, 0);
        double dvfb[3] = {0, 0, 0}, sdv2 = 0.0, dt = 0.0;
        double* dst = reinterpret_cast<double*>(cs + (k - 1));
        const auto put2 = [&](int i, double a, double b) { *reinterpret_cast<double2*>(dst + i) = double2{a, b}; };
        if (live) {
            const Imu pr = load_imu(im + k - 1, bg, ba);
            const Imu ic = load_imu(im + k, bg, ba);
            dt = ic.dt;
            double c1[3], c2[3], c3[3], dth[3];
            cross3(ic.dth, ic.dv, c1);
            cross3(pr.dth, ic.dv, c2);
            cross3(pr.dv, ic.dth, c3);
            for (int i = 0; i < 3; ++i) dvfb[i] = ic.dv[i] + 0.5 * c1[i] + 1.0 / 12.0 * (c2[i] + c3[i]);
            cross3(pr.dth, ic.dth, c1);
            for (int i = 0; i < 3; ++i) dth[i] = ic.dth[i] + 1.0 / 12.0 * c1[i];
            // the step's own increments go out first (short live ranges across
            // the scans; load_imu's dth / dv are already bias-compensated:
            // compensationBias)
            put2(0, dt, ic.dth[0]);
            put2(2, ic.dth[1], ic.dth[2]);
            put2(4, ic.dv[0], ic.dv[1]);
            sdv2 = ic.dv[2];
            qd = dq_from_rotvec_small(dth);
            if (EARTH) {
                const double dnn[3] = {-iewn[0] * dt, -iewn[1] * dt, -iewn[2] * dt};
                qnn = dq_from_rotvec_small(dnn);
            }
        }
        // the chains after step k: R_k = Rc qd_kc .. qd_k, L_k = qnn_k .. qnn_kc Lc
        // (steps past m carry the identity: they follow every live step)
        const dq R = dq_mul(Rc, wave_prefix_product<true>(qd));
        const dq dqt = dq_renorm(R);
        dq q;
        if constexpr (EARTH) {
            const dq L = dq_mul(wave_prefix_product<false>(qnn), Lc);
            q = dq_renorm(dq_mul(dq_mul(L, q0), R));
            Lc = dq_renorm(dq_readlane(L, 63));
        } else {
            q = dq_renorm(dq_mul(q0, R));
        }
        // the rotated terms of step k from the chain values after step k - 1
        // (lane k - 1, or the previous chunk's last step; q0 / identity at k = 1)
        const dq qprev = dq_wave_shr1(q, qlast), dprev = dq_wave_shr1(dqt, Rc);
        Rc = dq_readlane(dqt, 63);
        qlast = dq_readlane(q, 63);
        if (live) {
            double Rm[9], ra[3], rb[3];
            dq qc;
            if constexpr (!EARTH) {
                dq_rot(qprev, Rm);
                mv3(Rm, dvfb, ra);
                dq_rot(dprev, Rm);
                mv3(Rm, dvfb, rb);
                qc = dqt;
            } else {
                // ra = 0.5 (I + R(qnn)) R(qprev) dvfb, rb = R(qa dprev) dvfb, qc = qb dqt
                // (qa, qb: the Earth-rotation corrections at mid-step and at the
                // step's end, conjugated into the segment's start frame)
                double x[3], y[3];
                dq_rot(qprev, Rm);
                mv3(Rm, dvfb, x);
                dq_rot(qnn, Rm);
                mv3(Rm, x, y);
                for (int i = 0; i < 3; ++i) ra[i] = 0.5 * (x[i] + y[i]);
                const double sc = -(dtime - 0.5 * dt);
                const double dnn2[3] = {sc * iewn[0], sc * iewn[1], sc * iewn[2]};
                const dq qa = dq_mul(dq_mul(q0i, dq_from_rotvec_small(dnn2)), q0);
                dq_rot(dq_mul(qa, dprev), Rm);
                mv3(Rm, dvfb, rb);
                const double dnn3[3] = {-iewn[0] * dtime, -iewn[1] * dtime, -iewn[2] * dtime};
                const dq qb = dq_mul(dq_mul(q0i, dq_from_rotvec_small(dnn3)), q0);
                qc = dq_mul(qb, dqt);
            }
            put2(6, sdv2, qc.x);
            put2(8, qc.y, qc.z);
            put2(10, qc.w, ra[0]);
            put2(12, ra[1], ra[2]);
            put2(14, rb[0], rb[1]);
            put2(16, rb[2], 0.0);
        }
        if (k == m - 1) {  // the segment's last step
            dq_store(q, o->current.q);
            dq_store(dqt, o->delta.q);
            o->delta_time = dtime;
        }
    }
    if (lane == 0) {
        if (m <= 1) {
            dq_store(q0, o->current.q);
            dq_store(dq_make(1, 0, 0, 0), o->delta.q);
            o->delta_time = 0.0;
        }
        o->variant = EARTH ? GVX_PREINT_EARTH : GVX_PREINT_NORMAL;
        o->m = m;
        o->start_time = im[0].time;
        o->end_time = m > 1 ? im[m - 1].time : im[0].time;
        o->current.time = m > 1 ? im[m - 1].time : s0.time;
        o->delta.time = 0;
        for (int i = 0; i < 3; ++i) {
            o->current.bg[i] = s0.bg[i];
            o->current.ba[i] = s0.ba[i];
            o->delta.bg[i] = s0.bg[i];
            o->delta.ba[i] = s0.ba[i];
            o->gravity[i] = i == 2 ? prm.gravity : 0.0;
            o->iewn[i] = EARTH ? iewn_in[3 * seg + i] : 0.0;
        }
        dq_store(q0, o->q0);
    }
}

// The covariance pass (r05): 16 lanes per segment, 4 segments per one-wave
// workgroup; lane c owns column c of J and of P (P is symmetric, so also row c).
// Every 8 steps the lanes c < 8 of a segment's group form ONE step's record each
// into LDS (StepRec: Phi's blocks, W, the rotated increments, the lookups of
// Phi's row c); then the 8 steps run in sequence.  A step is branch-free up to
// its last assignment:
//   * its whole record is read into registers at once (the broadcast blocks, the
//     lane's row of Phi, the lane's W column of the Q term): one wait, not one
//     per mat-vec;
//   * G(:,c) = Phi P(:,c) is stored transposed -- lane c writes element i to
//     row i of the segment's LDS tile (sT, 18 doubles a row: rows 16-B aligned,
//     the 16 lanes' 8-byte stores contiguous and the b128 row reads of 16 lanes
//     on 16 distinct 4-bank windows), so lane c then reads row c, i.e.
//     K = G(c,:)^T, as seven ds_read_b128 + one b64 instead of fifteen
//     strided reads;
//   * K's Q terms (a W(:,c), the same fp64 adds as before) are LDS adds issued
//     after a wave fence, their operands formed before the stores (no LDS
//     round trip, no lgkmcnt(0) drain in the step);
//   * J <- Phi J runs between the stores and the reads;
//   * P'(:,c) = Phi K + a W phi_c (q_terms), assigned where the step is live.
// Steps past a segment's m (ragged batches: the wave runs to the longest of its
// four) read an identity record (dt = 0, f = 1, C = D = W = 0, M = I, a = b =
// 0), which leaves J, the sums and the record outputs unchanged; P keeps its
// value through the final assignment's predicate (an identity step would
// otherwise hand back P^T).  The operations and their order are those of
// preint_kernel (the one-phase form), so the two forms agree value for value
// (tests/test_ba_gpu.py::test_preint_two_phase_equals_one_phase).
// Reference: preintegration_earth.cc:266-303, preintegration_normal.cc:198-232
// (updateJacobianAndCovariance), preintegration_earth.cc:205-260 (the sums).
struct StepRec {
    double dt, f;             // PhiT's scalars (the layout of PhiT, so the step reads it in place)
    double C[9], D[9];        // Phi(3:6, 6:9), Phi(3:6, 12:15)
    double th[3], pad0;       // dtheta: Phi(6:9, 6:9) = I - skew(dtheta) (phi_mv_t forms its rows)
    double M[9], pad1;        // I - skew(dtheta), for lanes 6..8's row lookups
    double a[3], b[3];        // velocity / delta-velocity increments (before gravity / Coriolis)
    double pad2[4];
    // row c of Phi, read by lane c at a lane-dependent offset instead of selected:
    // S = {0,0,dt,0,0,f,0,0,-dt,0,0} (rows of dt I, f I, -dt I at 2-j, 5-j, 8-j),
    // S1 = {0,0,1,0,0} (rows of I), Z = zeros
    double S[11], S1[5], Z[3], pad;
};
static_assert(sizeof(Phi) == 29 * 8, "Phi is StepRec's prefix");
constexpr int SREC_DW = sizeof(StepRec) / 8;  // 64
constexpr int C16_CK = 6;   // steps per record chunk (one per lane c < 6 of a group)
constexpr int TS = 18;      // sT row stride (doubles): 16-B aligned rows, conflict-free b128 row reads
constexpr int TSEG = 288;   // sT doubles per segment: 15 rows of 18, padded to a multiple of 256 B
static_assert(TSEG >= 16 * TS - 2 && (TSEG * 8) % 256 == 0, "sT layout");
// records in LDS: RS doubles apart (528 B: the 8 lanes writing a chunk's records
// hit 8 distinct 4-bank windows instead of one, 8-way), segments SEGR doubles
// apart (36 banks: the broadcast b128 reads of two segments' lanes sharing a lane
// group do not collide).  PMC r05 v3: 39 % of the LDS cycles were bank conflicts.
constexpr int RS = SREC_DW + 2;
constexpr int SEGR = C16_CK * RS + 2;
static_assert((RS * 8) % 16 == 0 && (SEGR * 8) % 16 == 0, "16-B aligned records");
// the next chunk's CovIn records are staged by LDS-DMA (global_load_lds, 16 B a
// lane) while the current chunk's steps run: the record phase reads LDS, not
// HBM (the r05 v12 stamps put a chunk's record phase at ~8,800 cycles, most of
// it the global round trip and the rotated terms, now formed in the pre pass)
// One DMA instruction (64 lanes x 16 B) per segment: a segment's staging slot
// is 1 KB, its 6 records (864 B) in the first 54 pieces, so each instruction's
// source base and m are the segment's own (uniform, scalar registers)
constexpr int STG_SEG = 128;                                // doubles per segment slot
constexpr int STG_PIECES = C16_CK * COVIN_DW * 8 / 16;      // 16-B pieces staged per segment (54)
static_assert(STG_PIECES <= 64 && C16_CK * COVIN_DW <= STG_SEG, "a chunk's records fit one DMA instruction");
constexpr int STG_INS = 4;                                  // DMA instructions per chunk (one per segment)
// LDS per wave: 4 x 3,184 B of records + 4 x 2,304 B of transpose tiles + 4 x
// 864 B of staging = 25.4 KB, so the 1,312 waves of a 5,247-segment batch are
// resident at once (6 per CU)

// per segment group in the record region: A and X (15 x 15 each) and perm
constexpr int SI_GROUP_DW = 2 * NS * NS + 8;
constexpr int C16_LDS_REC = (4 * SEGR + 31) / 32 * 32, C16_LDS_T = 4 * TSEG, C16_LDS_STG = STG_INS * 128;
static_assert(4 * SI_GROUP_DW <= C16_LDS_REC + C16_LDS_T, "sqrt_info scratch fits the record + tile region");
static_assert(C16_LDS_REC % 32 == 0 && C16_LDS_T % 32 == 0, "256-B aligned sub-regions");

// The record of step k (k >= 1) of one segment from its staged CovIn (in LDS):
// cbb0 = -R(qc), Phi's blocks (C by skew's structure, fused), dtheta and the
// increments.  No W: gR (nacc I) gR^T of a rotation is nacc I up to rounding,
// which the step adds on P's diagonal (wdc, wq).
template <bool EARTH>
__device__ __forceinline__ void make_record(const gvx_imu_params& prm, const double* __restrict__ ci,
                                            double* __restrict__ dst) {
    // each field stored as it is formed (short live ranges: the step loop's J, P
    // and sums stay in registers across the record phase)
    const auto put2 = [&](int i, double x, double y) { *reinterpret_cast<double2*>(dst + i) = double2{x, y}; };
    constexpr int oC = offsetof(StepRec, C) / 8, oD = offsetof(StepRec, D) / 8, oM = offsetof(StepRec, M) / 8;
    constexpr int oA = offsetof(StepRec, a) / 8, oS = offsetof(StepRec, S) / 8;
    constexpr int oT = offsetof(StepRec, th) / 8;
    static_assert(oC == 2 && oD == 11 && oT == 20 && oM == 24 && oA == 34 && oS == 44 && sizeof(PhiT) == 24 * 8,
                  "record layout");
    constexpr int iDT = offsetof(CovIn, dt) / 8, iTH = offsetof(CovIn, sdth) / 8, iDV = offsetof(CovIn, sdv) / 8;
    constexpr int iQC = offsetof(CovIn, qc) / 8, iA = offsetof(CovIn, a) / 8, iB = offsetof(CovIn, b) / 8;
    const double dt = ci[iDT];
    const double f = 1 - dt / prm.corr_time;
    const double sdth[3] = {ci[iTH], ci[iTH + 1], ci[iTH + 2]};
    const double sdv[3] = {ci[iDV], ci[iDV + 1], ci[iDV + 2]};
    double cbb0[9];
    dq_rot(dq_load(ci + iQC), cbb0);
#pragma unroll
    for (int i = 0; i < 9; ++i) cbb0[i] = -cbb0[i];
    // C = cbb0 skew(dv), by skew's two non-zeros per column (a product and a fused
    // multiply-add per entry instead of mm3's three products against a zero)
    double S[9], C[9], M[9];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double* r = cbb0 + 3 * i;
        C[3 * i] = __builtin_fma(r[1], sdv[2], -(r[2] * sdv[1]));
        C[3 * i + 1] = __builtin_fma(r[2], sdv[0], -(r[0] * sdv[2]));
        C[3 * i + 2] = __builtin_fma(r[0], sdv[1], -(r[1] * sdv[0]));
    }
    skew(sdth, S);
#pragma unroll
    for (int i = 0; i < 9; ++i) M[i] = ((i % 4) == 0 ? 1.0 : 0.0) - S[i];
    // dt, f, C[0..8], D[0..8], M[0..8] (doubles 0..28), W (29..37), a (38..40), b (41..43)
    put2(0, dt, f);
#pragma unroll
    for (int i = 0; i < 8; i += 2) put2(oC + i, C[i], C[i + 1]);
    put2(oC + 8, C[8], cbb0[0] * dt);
#pragma unroll
    for (int i = 1; i < 9; i += 2) put2(oD + i, cbb0[i] * dt, cbb0[i + 1] * dt);
#pragma unroll
    for (int i = 0; i < 8; i += 2) put2(oM + i, M[i], M[i + 1]);
    // W = gR (nacc I) gR^T with gR = +-R(qc) a rotation: nacc I up to rounding
    // (1e-16), so the record carries no W; the step adds a nacc on P's diagonal
    // like the gyro and bias terms (covariance kernel, wdc and wq)
    put2(oM + 8, M[8], 0.0);
    put2(oT, sdth[0], sdth[1]);
    put2(oT + 2, sdth[2], 0.0);
    put2(oA, ci[iA], ci[iA + 1]);
    put2(oA + 2, ci[iA + 2], ci[iB]);
    put2(oA + 4, ci[iB + 1], ci[iB + 2]);
    // S = {0,0,dt,0,0,f,0,0,-dt,0,0}: its three step values (the constant rest
    // of S, S1 = {0,0,1,0,0}, Z = 0 and the pad are written once per slot,
    // record_constants: 10 b128 stores a record fewer)
    dst[oS + 2] = dt;
    dst[oS + 5] = f;
    dst[oS + 8] = -dt;
}

// the identity step (past a segment's m): Phi = I, W = 0, no increments
// (S's three step values and everything before S; the rest is record_constants')
__device__ __forceinline__ void identity_record(double* __restrict__ dst) {
    constexpr int oS = offsetof(StepRec, S) / 8;
    double w[oS];
#pragma unroll
    for (int i = 0; i < oS; ++i) w[i] = 0.0;
    w[offsetof(StepRec, f) / 8] = 1.0;
    w[offsetof(StepRec, M) / 8] = 1.0;
    w[offsetof(StepRec, M) / 8 + 4] = 1.0;
    w[offsetof(StepRec, M) / 8 + 8] = 1.0;
#pragma unroll
    for (int i = 0; i < oS; i += 2) *reinterpret_cast<double2*>(dst + i) = double2{w[i], w[i + 1]};
    dst[oS + 2] = 0.0;
    dst[oS + 5] = 1.0;
    dst[oS + 8] = 0.0;
}
// the constant part of a record slot's lookups: S = {0,0,*,0,0,*,0,0,*,0,0},
// S1 = {0,0,1,0,0}, Z = 0 and the pad, written once per slot before the steps
__device__ __forceinline__ void record_constants(double* __restrict__ dst) {
    constexpr int oS = offsetof(StepRec, S) / 8, oS1 = offsetof(StepRec, S1) / 8;
    static_assert(oS % 2 == 0 && SREC_DW - oS == 20, "S .. pad: 10 pairs");
#pragma unroll
    for (int i = oS; i < SREC_DW; i += 2)
        *reinterpret_cast<double2*>(dst + i) = double2{i == oS1 + 2 ? 1.0 : 0.0, i + 1 == oS1 + 2 ? 1.0 : 0.0};
}

// s_waitcnt vmcnt(0) (gfx9 encoding: expcnt and lgkmcnt left at their maxima)
constexpr int VMCNT0 = 0x0F70;

// 16 B per lane from global memory into LDS (lane l's piece at lds + 16 l):
// the LDS-DMA form of global_load_lds_dwordx4, issued from inline asm.  Through
// the builtin the compiler tracks the in-flight DMA as an LDS write and makes
// the next LDS access of the step loop wait for it (vmcnt(0): a full HBM round
// trip a chunk, r05 v17); hidden from it, the DMA is waited for only where the
// kernel says so (s_waitcnt vmcnt(0) before the staging is read).  Waits the
// compiler inserts for its own loads can only over-count an extra unknown
// operation, never under-count it.
__device__ __forceinline__ void dma16(const double* src, const double* lds) {
    typedef __attribute__((address_space(3))) const void* lptr;
    const uint32_t l = (uint32_t)(uintptr_t)(lptr)lds;
    uint32_t saved;  // m0 is reserved to the compiler: restored, not clobbered
    __asm__ volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(saved)
        : "v"(src), "s"(l)
        : "memory");
}

template <bool EARTH>
__global__ void __launch_bounds__(64, 2) preint_cov16_kernel(gvx_imu_params prm, int seg0, int seg_end,
                                                          const gvx_imu* __restrict__ imu,
                                                          const int32_t* __restrict__ seg_off,
                                                          const gvx_state* __restrict__ state0,
                                                          const double* __restrict__ iewn_in,
                                                          const CovIn* __restrict__ cin,
                                                          gvx_preint_result* __restrict__ out, double* __restrict__ pn) {
    // the kernel is written for ONE wave per workgroup: its LDS hand-overs are
    // wave fences (in-order LDS within a wave), and sqrt_info_group's barriers
    // are reached by every lane (dead groups factor the identity)
    constexpr int LANES = 16, SPWL = 64 / LANES;
    static_assert(SPWL * LANES == 64, "one wave per workgroup");
    // records | transpose tiles in one buffer (sqrt_info's scratch spans both
    // after the step loop); the DMA staging in its own: a distinct LDS object
    // lets the compiler see that the step loop's LDS reads do not alias the
    // in-flight DMA, so they do not wait for it (vmcnt)
    __shared__ __attribute__((aligned(256))) double sLds[C16_LDS_REC + C16_LDS_T];
    __shared__ __attribute__((aligned(16))) double sStg[C16_LDS_STG];  // the next chunk's CovIn records
    double* const sRec = sLds;
    const int lane = threadIdx.x;
    const int grp = lane / LANES, c = lane % LANES;
    const int wseg = seg0 + blockIdx.x * SPWL;  // the wave's first segment
    const int seg = wseg + grp;
    const bool live = seg < seg_end;
    const int b0 = live ? seg_off[seg] : 0;
    const int m = live ? seg_off[seg + 1] - b0 : 0;
    int mmax = m;
#pragma unroll
    for (int o = LANES; o < 64; o <<= 1) mmax = max(mmax, __shfl_xor(mmax, o));
    double* pns = (pn && live && EARTH) ? pn + (size_t)(b0 - seg) * 4 : nullptr;
    gvx_state s0{};
    double iewn[3] = {0, 0, 0};
    if (live) {
        s0 = state0[seg];
        if (EARTH)
            for (int i = 0; i < 3; ++i) iewn[i] = iewn_in[3 * seg + i];
    }
    double p[3], v[3], dp[3] = {0, 0, 0}, dv[3] = {0, 0, 0};
    for (int i = 0; i < 3; ++i) {
        p[i] = s0.p[i];
        v[i] = s0.v[i];
    }
    const double g3[3] = {0, 0, prm.gravity};
    const double nacc = prm.acc_vrw * prm.acc_vrw;
    const double ngyr = prm.gyr_arw * prm.gyr_arw;
    const double nbg = 2 * prm.gyr_bias_std * prm.gyr_bias_std / prm.corr_time;
    const double nba = 2 * prm.acc_bias_std * prm.acc_bias_std / prm.corr_time;
    const double g60 = EARTH ? -1.0 : 1.0;
    const double wg = (g60 * ngyr) * g60;
    // the diagonal Q term of lane c's row (W = nacc I, see make_record); lanes
    // 0..2 have none
    const double wdc = c < 3 ? 0.0 : (c < 6 ? nacc : (c < 9 ? wg : (c < 12 ? nbg : nba)));
    constexpr int oC = offsetof(StepRec, C) / 8, oD = offsetof(StepRec, D) / 8, oM = offsetof(StepRec, M) / 8;
    constexpr int oS = offsetof(StepRec, S) / 8, oS1 = offsetof(StepRec, S1) / 8, oZ = offsetof(StepRec, Z) / 8;
    constexpr int oA = offsetof(StepRec, a) / 8;
    // lane-dependent lookups into a record: row c of Phi (cols 3..14) and the W
    // column of lane c's Q adds (lanes 3..5; the others read a zero)
    const int ph3 = c < 3 ? oS + 2 - c : (c < 6 ? oS1 + 2 - (c - 3) : oZ);
    const int ph6 = (c >= 3 && c < 6) ? oC + 3 * (c - 3) : ((c >= 6 && c < 9) ? oM + 3 * (c - 6) : oZ);
    const int ph9 = (c >= 6 && c < 9) ? oS + 8 - (c - 6) : ((c >= 9 && c < 12) ? oS + 5 - (c - 9) : oZ);
    const int ph12 = (c >= 3 && c < 6) ? oD + 3 * (c - 3) : ((c >= 12 && c < NS) ? oS + 5 - (c - 12) : oZ);
    // lane c's W column (c mod 3): the Q adds of lanes 3..5 and q_terms' W phi_c(3:6)
    // (phi_c(3:6) has its one non-zero, dt for c < 3 or 1 for c < 6, at c mod 3)
    const int qw = c % 3;
    const int phs = ph3 + qw;
    const bool qdl = c >= 3 && c < NS;  // lanes with a diagonal Q add
    // lane c's W column (c mod 3) of q_terms: nacc at row c mod 3
    double wq[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) wq[i] = i == qw ? nacc : 0.0;
    double Jc[NS], Pc[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        Jc[i] = i == c ? 1.0 : 0.0;
        Pc[i] = 0.0;
    }
    double* const tile = sLds + C16_LDS_REC + grp * TSEG;
    // LDS-DMA of a chunk's CovIn records (steps kc .. kc + C16_CK - 1 of the four
    // segments) into sStg: 16-B piece pc of the wave's staging is piece pc % P of
    // segment pc / P's chunk (P = 54); pieces of steps past a segment's m (or of
    // dead groups) re-read a valid record and are never used
    // the four segments' first CovIn record and m (uniform: scalar registers;
    // per-lane copies kept across the step loop were spilled, and their
    // reloads serialised every record phase: 4,800 cycles, r05 v17 stamps)
    const int m0s = __builtin_amdgcn_readlane(m, 0), m1s = __builtin_amdgcn_readlane(m, LANES);
    const int m2s = __builtin_amdgcn_readlane(m, 2 * LANES), m3s = __builtin_amdgcn_readlane(m, 3 * LANES);
    const int wb = __builtin_amdgcn_readlane(b0, 0) - wseg;  // dead groups: record 0
    const int b1s = m1s > 0 ? __builtin_amdgcn_readlane(b0, LANES) - (wseg + 1) : 0;
    const int b2s = m2s > 0 ? __builtin_amdgcn_readlane(b0, 2 * LANES) - (wseg + 2) : 0;
    const int b3s = m3s > 0 ? __builtin_amdgcn_readlane(b0, 3 * LANES) - (wseg + 3) : 0;
    // piece `lane` of a slot: record (2 lane) / 18 of the chunk, double
    // (2 lane) % 18 inside it; records 0 .. m-2 hold steps 1 .. m-1
    const auto piece = [&](int kc, int bg, int mg) {
        const int rec = max(min(kc - 1 + (2 * lane) / COVIN_DW, mg - 2), 0);
        return reinterpret_cast<const double*>(cin + (bg + rec)) + (2 * lane) % COVIN_DW;
    };
    if (c < C16_CK) record_constants(sRec + grp * SEGR + c * RS);
    if (1 < mmax && lane < STG_PIECES) {
        dma16(piece(1, m0s > 0 ? wb : 0, m0s), sStg);
        dma16(piece(1, b1s, m1s), sStg + STG_SEG);
        dma16(piece(1, b2s, m2s), sStg + 2 * STG_SEG);
        dma16(piece(1, b3s, m3s), sStg + 3 * STG_SEG);
    }
    // pn rows (dt, p) of the chunk's steps: lane c < C16_CK keeps step kc + c's
    // and stores it during the next chunk's record phase, after that chunk's
    // DMA has been waited for (a store issued inside the step loop would hold up
    // the next chunk's vmcnt(0) wait by a full write round trip)
    double prow[4] = {0, 0, 0, 0};
    int prk = 0;  // the step prow belongs to (0: none)
    const auto store_prow = [&]() {
        if (pns && c < C16_CK && prk >= 1 && prk < m)
            *reinterpret_cast<double4*>(pns + 4 * (prk - 1)) = double4{prow[0], prow[1], prow[2], prow[3]};
    };
    // The previous chunk's pn rows, then the next chunk's DMA, every operand
    // formed first: the kernel is VGPR-bound and some operands are spilled, and
    // a reload issued after a DMA waits (vmcnt(0)) for that DMA's round trip
    // (r05 v17 stamps: 4,800 cycles a chunk when the four issues were
    // interleaved with reloads).
    const auto stage_and_store = [&](int kc) {
        const int kn = kc + C16_CK;
        const bool dma = kn < mmax && lane < STG_PIECES;
        const double* s0p = piece(kn, m0s > 0 ? wb : 0, m0s);
        const double* s1p = piece(kn, b1s, m1s);
        const double* s2p = piece(kn, b2s, m2s);
        const double* s3p = piece(kn, b3s, m3s);
        const bool st = pns && c < C16_CK && prk >= 1 && prk < m;
        double* pdst = st ? pns + 4 * (prk - 1) : pn;
        const double4 pv{prow[0], prow[1], prow[2], prow[3]};
        if (st) *reinterpret_cast<double4*>(pdst) = pv;
        __builtin_amdgcn_sched_barrier(0);
        if (dma) {
            dma16(s0p, sStg);
            dma16(s1p, sStg + STG_SEG);
            dma16(s2p, sStg + 2 * STG_SEG);
            dma16(s3p, sStg + 3 * STG_SEG);
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    for (int kc = 1; kc < mmax; kc += C16_CK) {
        // ---- this chunk's step records, one step per lane, from the staged CovIn ----
        // the chunk's DMA has landed (the intrinsic, not asm: the compiler then
        // knows nothing of its own is outstanding either, and puts no waits for
        // older reloads inside the step loop, where they would catch the next DMA)
        __builtin_amdgcn_s_waitcnt(VMCNT0);
        wave_lds_sync();
        if (c < C16_CK) {
            const int k = kc + c;
            double* dst = sRec + grp * SEGR + c * RS;
            if (k < m)
                make_record<EARTH>(prm, sStg + grp * STG_SEG + c * COVIN_DW, dst);
            else
                identity_record(dst);
        }
        // the staging is read: the next chunk's records land there while this
        // chunk's steps run
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stage_and_store(kc);
        prk = kc + c;
        wave_lds_sync();
        const int kend = min(kc + C16_CK, mmax);
        for (int k = kc; k < kend; ++k) {
            const bool act = k < m;
            const double* rw = sRec + grp * SEGR + (k - kc) * RS;
            // the record's Phi, increments and this lane's Q operands (one wait);
            // W and row c of Phi are read after the hand-over, where they are used
            const PhiT f = *reinterpret_cast<const PhiT*>(rw);
            double ra[3], rb[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                ra[i] = rw[oA + i];
                rb[i] = rw[oA + 3 + i];
            }
            const double sc = rw[phs];
            const double dt = f.dt;
            const double a = 0.5 * dt;
            // the velocity / position sums (integrationProcess, the order of preint_kernel)
            double dvel[3];
            if constexpr (!EARTH) {
#pragma unroll
                for (int i = 0; i < 3; ++i) dvel[i] = ra[i] + g3[i] * dt;
            } else {
                double cc3[3], dvcg[3];
                cross3(iewn, v, cc3);
#pragma unroll
                for (int i = 0; i < 3; ++i) dvcg[i] = (g3[i] - 2.0 * cc3[i]) * dt;
#pragma unroll
                for (int i = 0; i < 3; ++i) dvel[i] = ra[i] + dvcg[i];
            }
#pragma unroll
            for (int i = 0; i < 3; ++i) p[i] += dt * v[i] + 0.5 * dt * dvel[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) v[i] += dvel[i];
            if (pns && k - kc == c) {
                prow[0] = dt;
                prow[1] = p[0];
                prow[2] = p[1];
                prow[3] = p[2];
            }
#pragma unroll
            for (int i = 0; i < 3; ++i) dp[i] += dt * dv[i] + 0.5 * dt * rb[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) dv[i] += rb[i];
            // G(:,c) = Phi P(:,c), stored transposed (element i to row i); lane 15
            // writes column 15, which no row read uses
            double y[NS];
            phi_mv_t(f, Pc, y);
#pragma unroll
            for (int i = 0; i < NS; ++i) tile[i * TS + c] = y[i];
            // K's Q term: a w_c onto the diagonal of row c (lanes 3..14; W = nacc I,
            // so lanes 3..5 add a nacc there) -- after every lane's stores
            const double qdg = a * wdc;
            wave_lds_sync();
            if (qdl) __hip_atomic_fetch_add(&tile[c * TS + c], qdg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            wave_lds_sync();
            // K = row c of the tile = G(c,:)^T + a W(:,c) (row 15 is padding) and
            // row c of Phi, cols 6..14; issued before J's update, which runs
            // while they land (sched_barrier: the compiler would sink it)
            double K[NS], ph[NS];
#pragma unroll
            for (int i = 0; i < NS; ++i) K[i] = tile[c * TS + i];
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                ph[6 + b] = rw[ph6 + b];
                ph[9 + b] = rw[ph9 + b];
                ph[12 + b] = rw[ph12 + b];
            }
            __builtin_amdgcn_sched_barrier(0);
            phi_mv_t(f, Jc, y);
#pragma unroll
            for (int i = 0; i < NS; ++i) Jc[i] = y[i];
            __builtin_amdgcn_sched_barrier(0);
            if (act) {
                phi_mv_t(f, K, y);
#pragma unroll
                for (int i = 0; i < 3; ++i) Pc[i] = y[i];
                // q_terms with W phi_c(3:6) = sc W(:, c mod 3) (the other two terms
                // of the sum are exact zeros)
#pragma unroll
                for (int i = 0; i < 3; ++i) Pc[3 + i] = __builtin_fma(a, wq[i] * sc, y[3 + i]);
                const double ag = a * wg, abg = a * nbg, aba = a * nba;
#pragma unroll
                for (int i = 6; i < NS; ++i) Pc[i] = __builtin_fma(i < 9 ? ag : (i < 12 ? abg : aba), ph[i], y[i]);
            }
            wave_lds_sync();  // the next step's stores after this step's reads
        }
    }
    store_prow();
    gvx_preint_result* o = out + seg;
    if (live && c < NS) {
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            o->jacobian[i * NS + c] = Jc[i];
            o->covariance[c * NS + i] = Pc[i];
        }
    }
    if (live && c == 0)
        for (int i = 0; i < 3; ++i) {
            o->current.p[i] = p[i];
            o->current.v[i] = v[i];
            o->delta.p[i] = dp[i];
            o->delta.v[i] = dv[i];
        }
    // sqrt_information_ from P while it is in registers, in the record region
    // (the same function as factors.hip sqrt_info_kernel, same bits): no extra
    // launch, no read-back of the covariance.  Dead groups factor the identity
    // and store nothing, so every lane reaches every barrier.
    wave_lds_sync();  // the last step's record reads are done
    double* A = sRec + grp * SI_GROUP_DW;
    double* X = A + NS * NS;
    int* perm = reinterpret_cast<int*>(X + NS * NS);
    if (c < NS) {
#pragma unroll
        for (int i = 0; i < NS; ++i) A[c * NS + i] = live ? Pc[i] : (i == c ? 1.0 : 0.0);
    }
    sqrt_info_group(A, X, perm, c, live ? o->sqrt_info : nullptr);
}

}  // namespace

hipError_t launch_preint(gvx_ctx* c, int variant, const gvx_imu_params& prm, int n_seg,
                         const gvx_imu* imu, const int32_t* seg_off, const gvx_state* state0,
                         const double* iewn, gvx_preint_result* out, double* pn, bool* sqrt_info_done) {
    if (sqrt_info_done) *sqrt_info_done = false;
    if (n_seg <= 0) return hipSuccess;
    // Two-launch form when the per-step scratch can be sized without a round
    // trip: the IMU allocation bounds the number of samples
    // (hipMemGetAddressRange).  A pointer into a large pooled block bounds nothing
    // useful: above 1 GiB of scratch the single kernel runs.
    // gvx_set_preint_path(GVX_PREINT_PATH_ONEPHASE) forces it (A/B and the parity
    // test of the two forms).
    hipDeviceptr_t base = nullptr;
    size_t range = 0;
    if (c->preint_path != GVX_PREINT_PATH_ONEPHASE &&
        hipMemGetAddressRange(&base, &range, (hipDeviceptr_t)imu) == hipSuccess && range > 0) {
        const size_t samples = (reinterpret_cast<const char*>(base) + range - reinterpret_cast<const char*>(imu)) /
                               sizeof(gvx_imu);
        const size_t bytes = samples * STEP_SCRATCH;
        char* d = bytes <= (size_t(1) << 30) ? (char*)scratch(c, "preint_steps", bytes) : nullptr;
        if (d) {
            const CovIn* ci = reinterpret_cast<CovIn*>(d);
            const bool earth = variant == GVX_PREINT_EARTH;
            // the per-step terms and the quaternion chains (wave scans) of
            // segments [s0, s1), then their covariance pass (sqrt_info in its
            // epilogue)
            const auto pre = [&](hipStream_t st, int s0, int s1) {
                hipLaunchKernelGGL(earth ? preint_pre_kernel<true> : preint_pre_kernel<false>, dim3(s1 - s0), dim3(64),
                                   0, st, s0, imu, seg_off, state0, iewn, (CovIn*)ci, prm, out);
            };
            const auto cov = [&](hipStream_t st, int s0, int s1) {
                hipLaunchKernelGGL(earth ? preint_cov16_kernel<true> : preint_cov16_kernel<false>,
                                   dim3((s1 - s0 + 3) / 4), dim3(64), 0, st, prm, s0, s1, imu, seg_off, state0, iewn,
                                   ci, out, pn);
            };
            // (r05 v15: splitting a batch in two, the first half's covariance pass
            // on a second stream beside the second half's pre pass, was 4 %
            // slower: the covariance waves are not latency-bound enough to share)
            pre(c->stream, 0, n_seg);
            cov(c->stream, 0, n_seg);
            if (sqrt_info_done) *sqrt_info_done = true;
            return hipGetLastError();
        }
    }
    (void)hipGetLastError();  // a failed range query is not an error of this call
    hipLaunchKernelGGL(preint_kernel, dim3((n_seg + SPW - 1) / SPW), dim3(64), 0, c->stream, variant, prm, n_seg, imu,
                       seg_off, state0, iewn, out, pn);
    return hipGetLastError();
}

}  // namespace gvx
