// ins.hip -- batched INS mechanization for gfx950 (fp64): the chain
// MISC::insMechanization(imu[k-1], imu[k], state), k = 1 .. m-1
// (/root/reference/ic_gvins/ic_gvins/misc.cc:174-229), as redoInsMechanization
// (:231-284) runs it over the INS window after every optimisation and the
// fusion thread runs it per IMU sample (ic_gvins.cc:304-310).
//
// One 64-lane wavefront per chain.  The terms of a step that do not depend on
// the recursion -- bias compensation (biases are constant along a chain),
// two-sample sculling / coning, rotvec2quaternion of dtheta and of -iewn dt --
// are computed for 64 steps at once, one step per lane, into LDS; the
// sequential part then only runs the cheap state update (rotation matrices,
// quaternion products, one normalisation).  Every expression follows the CPU
// restatement (oracle/ins.c) in order; states match it within the fp64 parity
// bound (ocml vs glibc sin/cos only).
#include <hip/hip_runtime.h>

#include "dmath.h"
#include "gvx_internal.h"

namespace gvx {

namespace {

struct InsStep {
    double dt, time;
    double dvfb[3];
    double qd[4];   // rotvec2quaternion(dtheta + coning)
    double qnn[4];  // Earth: rotvec2quaternion(-iewn dt)
    double m1[9];   // Earth: 0.5 (I + R(qnn)), also independent of the recursion
};
constexpr int STEP_DW = sizeof(InsStep) / 8;
constexpr int CHUNK = 64;

__device__ __forceinline__ void put_state(gvx_state* o, const gvx_state& s) {
    // lane 0 only: the state is wave-uniform
    o->time = s.time;
    for (int i = 0; i < 3; ++i) {
        o->p[i] = s.p[i];
        o->v[i] = s.v[i];
        o->bg[i] = s.bg[i];
        o->ba[i] = s.ba[i];
    }
    for (int i = 0; i < 4; ++i) o->q[i] = s.q[i];
}

__global__ void __launch_bounds__(64) ins_kernel(gvx_ins_config cfg, int n_chain, const gvx_imu* __restrict__ imu,
                                                 const int32_t* __restrict__ off, const gvx_state* __restrict__ state0,
                                                 gvx_state* __restrict__ states) {
    __shared__ double sst[CHUNK][STEP_DW];
    const int c = blockIdx.x;
    if (c >= n_chain) return;
    const int lane = threadIdx.x;
    const int b0 = off[c], m = off[c + 1] - b0;
    const gvx_imu* im = imu + b0;
    gvx_state* out = states + b0;
    gvx_state s = state0[c];
    const bool earth = cfg.iswithearth != 0;
    if (m > 0 && lane == 0) put_state(out, s);
    for (int kc = 1; kc < m; kc += CHUNK) {
        {
            const int k = kc + lane;
            if (k < m) {
                const gvx_imu& pr = im[k - 1];
                const gvx_imu& cu = im[k];
                double ct[3], cv[3], pt[3], pv[3];
                for (int i = 0; i < 3; ++i) {
                    ct[i] = cu.dtheta[i] - cu.dt * s.bg[i];
                    cv[i] = cu.dvel[i] - cu.dt * s.ba[i];
                    pt[i] = pr.dtheta[i] - pr.dt * s.bg[i];
                    pv[i] = pr.dvel[i] - pr.dt * s.ba[i];
                }
                InsStep st;
                st.dt = cu.dt;
                st.time = cu.time;
                double c1[3], c2[3], c3[3], dth[3];
                cross3(ct, cv, c1);
                cross3(pt, cv, c2);
                cross3(pv, ct, c3);
                for (int i = 0; i < 3; ++i) st.dvfb[i] = cv[i] + 0.5 * c1[i] + 1.0 / 12.0 * (c2[i] + c3[i]);
                cross3(pt, ct, c1);
                for (int i = 0; i < 3; ++i) dth[i] = ct[i] + 1.0 / 12.0 * c1[i];
                dq_store(dq_from_rotvec(dth), st.qd);
                if (earth) {
                    const double dnn[3] = {-cfg.iewn[0] * st.dt, -cfg.iewn[1] * st.dt, -cfg.iewn[2] * st.dt};
                    const dq qnn = dq_from_rotvec(dnn);
                    dq_store(qnn, st.qnn);
                    double Rnn[9];
                    dq_rot(qnn, Rnn);
                    for (int i = 0; i < 9; ++i) st.m1[i] = 0.5 * (((i % 4) == 0 ? 1.0 : 0.0) + Rnn[i]);
                }
                const double* w = reinterpret_cast<const double*>(&st);
                for (int i = 0; i < STEP_DW; ++i) sst[lane][i] = w[i];
            }
        }
        __syncthreads();
        const int kend = min(kc + CHUNK, m);
        for (int k = kc; k < kend; ++k) {
            const InsStep& st = *reinterpret_cast<const InsStep*>(sst[k - kc]);
            const double dt = st.dt;
            s.time = st.time;
            double dvel[3], Rq[9];
            dq q = dq_load(s.q);
            if (earth) {
                double cr[3], dvcg[3], M1[9];
                cross3(cfg.iewn, s.v, cr);
                for (int i = 0; i < 3; ++i) dvcg[i] = (cfg.gravity[i] - 2.0 * cr[i]) * dt;
                const dq qnn = dq_load(st.qnn);
                dq_rot(q, Rq);
                mm3(st.m1, Rq, M1);
                mv3(M1, st.dvfb, dvel);
                for (int i = 0; i < 3; ++i) dvel[i] = dvel[i] + dvcg[i];
                q = dq_normalized(dq_mul(dq_mul(qnn, q), dq_load(st.qd)));
            } else {
                dq_rot(q, Rq);
                mv3(Rq, st.dvfb, dvel);
                for (int i = 0; i < 3; ++i) dvel[i] = dvel[i] + cfg.gravity[i] * dt;
                q = dq_normalized(dq_mul(q, dq_load(st.qd)));
            }
            dq_store(q, s.q);
            for (int i = 0; i < 3; ++i) s.p[i] += dt * s.v[i] + 0.5 * dt * dvel[i];
            for (int i = 0; i < 3; ++i) s.v[i] += dvel[i];
            if (lane == 0) put_state(out + k, s);
        }
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_ins(gvx_ctx* c, const gvx_ins_config& cfg, int n_chain, const gvx_imu* imu, const int32_t* off,
                      const gvx_state* state0, gvx_state* states) {
    if (n_chain <= 0) return hipSuccess;
    hipLaunchKernelGGL(ins_kernel, dim3(n_chain), dim3(64), 0, c->stream, cfg, n_chain, imu, off, state0, states);
    return hipGetLastError();
}

}  // namespace gvx
