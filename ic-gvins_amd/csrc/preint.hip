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
// rotation-vector exponentials.
#include <hip/hip_runtime.h>

#include "dmath.h"
#include "gvx_internal.h"

namespace gvx {

namespace {

constexpr int NS = 15;

struct Imu {
    double dt, dth[3], dv[3], time;
};

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

// The non-zero structure of Phi for one step (updateJacobianAndCovariance).
struct Phi {
    double dt, ndt, f;   // dt, -dt, 1 - dt/corr_time
    double C[9];         // Phi(3:6, 6:9) = cbb0 * skew(dvel)
    double D[9];         // Phi(3:6, 12:15) = cbb0 * dt
    double M[9];         // Phi(6:9, 6:9) = I - skew(dtheta)
    double gR[9];        // gt(3:6, 3:6)
    double g60;          // gt(6:9, 0:3) diagonal
    double N[12];        // noise diagonal
};

// (Phi * X)[i][j], X row-major 15x15 (k ascending over Phi's row i non-zeros)
__device__ __forceinline__ double phi_left(const Phi& f, const double* X, int i, int j) {
    if (i < 3) return X[i * NS + j] + f.dt * X[(3 + i) * NS + j];
    if (i < 6) {
        const int a = i - 3;
        double s = X[i * NS + j];
        s = s + f.C[3 * a] * X[6 * NS + j];
        s = s + f.C[3 * a + 1] * X[7 * NS + j];
        s = s + f.C[3 * a + 2] * X[8 * NS + j];
        s = s + f.D[3 * a] * X[12 * NS + j];
        s = s + f.D[3 * a + 1] * X[13 * NS + j];
        s = s + f.D[3 * a + 2] * X[14 * NS + j];
        return s;
    }
    if (i < 9) {
        const int a = i - 6;
        double s = f.M[3 * a] * X[6 * NS + j];
        s = s + f.M[3 * a + 1] * X[7 * NS + j];
        s = s + f.M[3 * a + 2] * X[8 * NS + j];
        s = s + f.ndt * X[(9 + a) * NS + j];
        return s;
    }
    return f.f * X[i * NS + j];
}

// (X * Phi^T)[i][j] = sum_k X[i][k] Phi[j][k]
__device__ __forceinline__ double phi_right(const Phi& f, const double* X, int i, int j) {
    const double* x = X + i * NS;
    if (j < 3) return x[j] + x[3 + j] * f.dt;
    if (j < 6) {
        const int a = j - 3;
        double s = x[j];
        s = s + x[6] * f.C[3 * a];
        s = s + x[7] * f.C[3 * a + 1];
        s = s + x[8] * f.C[3 * a + 2];
        s = s + x[12] * f.D[3 * a];
        s = s + x[13] * f.D[3 * a + 1];
        s = s + x[14] * f.D[3 * a + 2];
        return s;
    }
    if (j < 9) {
        const int a = j - 6;
        double s = x[6] * f.M[3 * a];
        s = s + x[7] * f.M[3 * a + 1];
        s = s + x[8] * f.M[3 * a + 2];
        s = s + x[9 + a] * f.ndt;
        return s;
    }
    return x[j] * f.f;
}

// Phi[i][k] (dense accessor used by Qk)
__device__ __forceinline__ double phi_at(const Phi& f, int i, int k) {
    if (i < 3) return k == i ? 1.0 : (k == 3 + i ? f.dt : 0.0);
    if (i < 6) {
        const int a = i - 3;
        if (k == i) return 1.0;
        if (k >= 6 && k < 9) return f.C[3 * a + k - 6];
        if (k >= 12) return f.D[3 * a + k - 12];
        return 0.0;
    }
    if (i < 9) {
        const int a = i - 6;
        if (k >= 6 && k < 9) return f.M[3 * a + k - 6];
        if (k == 9 + a) return f.ndt;
        return 0.0;
    }
    return k == i ? f.f : 0.0;
}

// t2[i][c] = (Phi * gt)[i][c] * N[c]
__device__ __forceinline__ double t2_at(const Phi& f, int i, int c) {
    double t1;
    if (c < 3)
        t1 = phi_at(f, i, 6 + c) * f.g60;
    else if (c < 6) {
        const int b = c - 3;
        t1 = phi_at(f, i, 3) * f.gR[b];
        t1 = t1 + phi_at(f, i, 4) * f.gR[3 + b];
        t1 = t1 + phi_at(f, i, 5) * f.gR[6 + b];
    } else if (c < 9)
        t1 = phi_at(f, i, 9 + c - 6) * 1.0;
    else
        t1 = phi_at(f, i, 12 + c - 9) * 1.0;
    return t1 * f.N[c];
}

// Qk[i][j] = 0.5 dt (Phi G N G^T + G N G^T Phi^T)[i][j]
__device__ double qk_at(const Phi& f, int i, int j) {
    // A = ((Phi gt) N) gt^T
    double A;
    if (j < 3)
        A = 0.0;
    else if (j < 6) {
        const int a = j - 3;
        A = t2_at(f, i, 3) * f.gR[3 * a];
        A = A + t2_at(f, i, 4) * f.gR[3 * a + 1];
        A = A + t2_at(f, i, 5) * f.gR[3 * a + 2];
    } else if (j < 9)
        A = t2_at(f, i, j - 6) * f.g60;
    else
        A = t2_at(f, i, j - 3) * 1.0;
    // B = ((gt N) gt^T) Phi^T ; G = (gt N) gt^T is block diagonal
    double B;
    if (i < 3)
        B = 0.0;
    else if (i < 6) {
        const int a = i - 3;
        double Gr[3];
        for (int b = 0; b < 3; ++b) {
            double g = (f.gR[3 * a] * f.N[3]) * f.gR[3 * b];
            g = g + (f.gR[3 * a + 1] * f.N[4]) * f.gR[3 * b + 1];
            g = g + (f.gR[3 * a + 2] * f.N[5]) * f.gR[3 * b + 2];
            Gr[b] = g;
        }
        B = Gr[0] * phi_at(f, j, 3);
        B = B + Gr[1] * phi_at(f, j, 4);
        B = B + Gr[2] * phi_at(f, j, 5);
    } else if (i < 9) {
        const double g = (f.g60 * f.N[i - 6]) * f.g60;
        B = g * phi_at(f, j, i);
    } else {
        const double g = (1.0 * f.N[i - 3]) * 1.0;
        B = g * phi_at(f, j, i);
    }
    return 0.5 * f.dt * (A + B);
}

__global__ void __launch_bounds__(64) preint_kernel(int variant, gvx_imu_params prm, int n_seg,
                                                    const gvx_imu* __restrict__ imu,
                                                    const int32_t* __restrict__ seg_off,
                                                    const gvx_state* __restrict__ state0,
                                                    const double* __restrict__ iewn_in,
                                                    gvx_preint_result* __restrict__ out,
                                                    double* __restrict__ pn) {
    __shared__ double sJ[2][NS * NS];
    __shared__ double sP[NS * NS];
    __shared__ double sG[NS * NS];
    const int seg = blockIdx.x;
    if (seg >= n_seg) return;
    const int lane = threadIdx.x;
    const int b0 = seg_off[seg], m = seg_off[seg + 1] - b0;
    const gvx_imu* im = imu + b0;
    double* pns = pn ? pn + (size_t)(b0 - seg) * 4 : nullptr;
    const bool earth = variant == GVX_PREINT_EARTH;

    // ---- constructor: resetState(state, NUM_STATE) + setNoiseMatrix ----
    gvx_state cur = state0[seg];
    double dp[3] = {0, 0, 0}, dv[3] = {0, 0, 0};
    dq dqt = dq_make(1, 0, 0, 0);
    double bg[3], ba[3];
    for (int i = 0; i < 3; ++i) {
        bg[i] = cur.bg[i];
        ba[i] = cur.ba[i];
    }
    const dq q0 = dq_load(cur.q);
    double iewn[3] = {0, 0, 0};
    if (earth)
        for (int i = 0; i < 3; ++i) iewn[i] = iewn_in[3 * seg + i];
    const double g3[3] = {0, 0, prm.gravity};
    double delta_time = 0.0;
    Phi f;
    {
        const double nv[4] = {prm.gyr_arw * prm.gyr_arw, prm.acc_vrw * prm.acc_vrw,
                              2 * prm.gyr_bias_std * prm.gyr_bias_std / prm.corr_time,
                              2 * prm.acc_bias_std * prm.acc_bias_std / prm.corr_time};
        for (int b = 0; b < 4; ++b)
            for (int i = 0; i < 3; ++i) f.N[3 * b + i] = nv[b];
    }
    for (int e = lane; e < NS * NS; e += 64) {
        const int i = e / NS, j = e - i * NS;
        sJ[0][e] = i == j ? 1.0 : 0.0;
        sP[e] = 0.0;
    }
    int jb = 0;
    __syncthreads();

    for (int k = 1; k < m; ++k) {
        const Imu pre = load_imu(im + k - 1, bg, ba);
        const Imu ic = load_imu(im + k, bg, ba);
        const double dt = ic.dt;
        delta_time += dt;
        // dvfb: two-sample sculling (preintegration_base.cc:47-48)
        double c1[3], c2[3], c3[3], dvfb[3], dth[3];
        cross3(ic.dth, ic.dv, c1);
        cross3(pre.dth, ic.dv, c2);
        cross3(pre.dv, ic.dth, c3);
        for (int i = 0; i < 3; ++i) dvfb[i] = ic.dv[i] + 0.5 * c1[i] + 1.0 / 12.0 * (c2[i] + c3[i]);
        cross3(pre.dth, ic.dth, c1);
        for (int i = 0; i < 3; ++i) dth[i] = ic.dth[i] + 1.0 / 12.0 * c1[i];
        const dq qd = dq_from_rotvec(dth);
        double R[9], dvel[3];
        double cbb0[9];
        if (!earth) {
            dq_rot(dq_load(cur.q), R);
            mv3(R, dvfb, dvel);
            for (int i = 0; i < 3; ++i) dvel[i] = dvel[i] + g3[i] * dt;
            for (int i = 0; i < 3; ++i) cur.p[i] += dt * cur.v[i] + 0.5 * dt * dvel[i];
            for (int i = 0; i < 3; ++i) cur.v[i] += dvel[i];
            dq_store(dq_normalized(dq_mul(dq_load(cur.q), qd)), cur.q);
            dq_rot(dqt, R);
            mv3(R, dvfb, dvel);
            for (int i = 0; i < 3; ++i) dp[i] += dt * dv[i] + 0.5 * dt * dvel[i];
            for (int i = 0; i < 3; ++i) dv[i] += dvel[i];
            dqt = dq_normalized(dq_mul(dqt, qd));
            dq_rot(dqt, R);
            for (int i = 0; i < 9; ++i) {
                cbb0[i] = -R[i];
                f.gR[i] = R[i];
            }
            f.g60 = 1.0;
        } else {
            double c[3], dvcg[3];
            cross3(iewn, cur.v, c);
            for (int i = 0; i < 3; ++i) dvcg[i] = (g3[i] - 2.0 * c[i]) * dt;
            const double dnn[3] = {-iewn[0] * dt, -iewn[1] * dt, -iewn[2] * dt};
            const dq qnn = dq_from_rotvec(dnn);
            double Rnn[9], M1[9];
            dq_rot(qnn, Rnn);
            for (int i = 0; i < 9; ++i) M1[i] = 0.5 * (((i % 4) == 0 ? 1.0 : 0.0) + Rnn[i]);
            dq_rot(dq_load(cur.q), R);
            mm3(M1, R, M1);
            mv3(M1, dvfb, dvel);
            for (int i = 0; i < 3; ++i) dvel[i] = dvel[i] + dvcg[i];
            for (int i = 0; i < 3; ++i) cur.p[i] += dt * cur.v[i] + 0.5 * dt * dvel[i];
            for (int i = 0; i < 3; ++i) cur.v[i] += dvel[i];
            if (pns && lane == 0) {
                pns[4 * (k - 1)] = dt;
                pns[4 * (k - 1) + 1] = cur.p[0];
                pns[4 * (k - 1) + 2] = cur.p[1];
                pns[4 * (k - 1) + 3] = cur.p[2];
            }
            dq_store(dq_normalized(dq_mul(dq_mul(qnn, dq_load(cur.q)), qd)), cur.q);
            const double sc = -(delta_time - 0.5 * dt);
            const double dnn2[3] = {sc * iewn[0], sc * iewn[1], sc * iewn[2]};
            const dq q0i = dq_inv(q0);
            dq qm = dq_mul(dq_mul(dq_mul(q0i, dq_from_rotvec(dnn2)), q0), dqt);
            dq_rot(qm, R);
            mv3(R, dvfb, dvel);
            for (int i = 0; i < 3; ++i) dp[i] += dt * dv[i] + 0.5 * dt * dvel[i];
            for (int i = 0; i < 3; ++i) dv[i] += dvel[i];
            dqt = dq_normalized(dq_mul(dqt, qd));
            // updateJacobianAndCovariance (preintegration_earth.cc:266-303)
            const double dnn3[3] = {-iewn[0] * delta_time, -iewn[1] * delta_time, -iewn[2] * delta_time};
            qm = dq_mul(dq_mul(dq_mul(q0i, dq_from_rotvec(dnn3)), q0), dqt);
            dq_rot(qm, R);
            for (int i = 0; i < 9; ++i) {
                cbb0[i] = -R[i];
                f.gR[i] = cbb0[i];
            }
            f.g60 = -1.0;
        }
        cur.time = ic.time;
        // Phi blocks
        double S[9];
        skew(ic.dv, S);
        mm3(cbb0, S, f.C);
        for (int i = 0; i < 9; ++i) f.D[i] = cbb0[i] * dt;
        skew(ic.dth, S);
        for (int i = 0; i < 9; ++i) f.M[i] = ((i % 4) == 0 ? 1.0 : 0.0) - S[i];
        f.dt = dt;
        f.ndt = -dt;
        f.f = 1 - dt / prm.corr_time;

        // J <- Phi J (into the other buffer); G <- Phi P
        const double* Jc = sJ[jb];
        double* Jn = sJ[jb ^ 1];
        for (int e = lane; e < NS * NS; e += 64) {
            const int i = e / NS, j = e - i * NS;
            Jn[e] = phi_left(f, Jc, i, j);
            sG[e] = phi_left(f, sP, i, j);
        }
        __syncthreads();
        for (int e = lane; e < NS * NS; e += 64) {
            const int i = e / NS, j = e - i * NS;
            sP[e] = phi_right(f, sG, i, j) + qk_at(f, i, j);
        }
        jb ^= 1;
        __syncthreads();
    }

    // ---- outputs ----
    gvx_preint_result* o = out + seg;
    for (int e = lane; e < NS * NS; e += 64) {
        o->jacobian[e] = sJ[jb][e];
        o->covariance[e] = sP[e];
    }
    if (lane == 0) {
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

}  // namespace

hipError_t launch_preint(gvx_ctx* c, int variant, const gvx_imu_params& prm, int n_seg,
                         const gvx_imu* imu, const int32_t* seg_off, const gvx_state* state0,
                         const double* iewn, gvx_preint_result* out, double* pn) {
    if (n_seg <= 0) return hipSuccess;
    hipLaunchKernelGGL(preint_kernel, dim3(n_seg), dim3(64), 0, c->stream, variant, prm, n_seg, imu,
                       seg_off, state0, iewn, out, pn);
    return hipGetLastError();
}

}  // namespace gvx
