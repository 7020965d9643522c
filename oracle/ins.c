/*
 * ins.c -- CPU restatement of the INS mechanization and the IMU-series
 * extraction around the preintegration (TEST INFRASTRUCTURE ONLY; see
 * gvx_oracle.h).  Paths relative to /root/reference/ic_gvins/ic_gvins/.
 *
 *   orc_ins_mechanization   MISC::insMechanization (misc.cc:174-229): bias
 *                           compensation, two-sample sculling / coning, then
 *                           Earth (Coriolis + gravity, qnn * q * q(dtheta)) or
 *                           plain (q * q(dtheta)) propagation; p uses the mean
 *                           velocity, v is updated last.  iswithscale is false in
 *                           the reference (ic_gvins.cc:116) and not restated.
 *   orc_ins_propagate       the chain insMechanization(imu[k-1], imu[k], state),
 *                           k = 1 .. m-1 (redoInsMechanization's loop,
 *                           misc.cc:269-275, and the fusion thread's per-sample
 *                           call, ic_gvins.cc:310).
 *   orc_ins_window_index    MISC::getInsWindowIndex (misc.cc:40-83): the first
 *                           index whose time is > t (binary search, 0 = none).
 *   orc_imu_interpolation   MISC::imuInterpolation (misc.cc:311-328) and
 *   orc_need_interpolation  MISC::isNeedInterpolation (misc.cc:286-309).
 *   orc_redo_ins_mechanization  MISC::redoInsMechanization (misc.cc:231-284)
 *                           without the final pop_front (the caller trims).
 *   orc_imu_series_from_to  MISC::getImuSeriesFromTo (misc.cc:330-384).
 * Eigen expressions are evaluated left to right without FMA contraction, the
 * 0.5 (I + Rnn) Rq product into a temporary first (as Eigen evaluates a nested
 * product).  Parity unpinned against the reference binaries (Eigen absent);
 * pinned by closed forms in tests/test_oracle_ins.py.
 */
#include <string.h>

#include "gvx_oracle.h"
#include "orc_math.h"

#define MIN_TIME_INTERVAL 0.0001 /* MISC::MINIMUM_TIME_INTERVAL, misc.h:72 */

void orc_ins_mechanization(const orc_ins_config* cfg, const orc_imu* pre, const orc_imu* cur, orc_state* s) {
    orc_imu c2 = *cur, p2 = *pre;
    for (int i = 0; i < 3; i++) {
        c2.dtheta[i] = cur->dtheta[i] - cur->dt * s->bg[i];
        c2.dvel[i] = cur->dvel[i] - cur->dt * s->ba[i];
        p2.dtheta[i] = pre->dtheta[i] - pre->dt * s->bg[i];
        p2.dvel[i] = pre->dvel[i] - pre->dt * s->ba[i];
    }
    const double dt = cur->dt;
    s->time = cur->time;
    double c1[3], cc2[3], c3[3], dvfb[3], dth[3];
    v3_cross(c2.dtheta, c2.dvel, c1);
    v3_cross(p2.dtheta, c2.dvel, cc2);
    v3_cross(p2.dvel, c2.dtheta, c3);
    for (int i = 0; i < 3; i++) dvfb[i] = c2.dvel[i] + 0.5 * c1[i] + 1.0 / 12.0 * (cc2[i] + c3[i]);
    v3_cross(p2.dtheta, c2.dtheta, c1);
    for (int i = 0; i < 3; i++) dth[i] = c2.dtheta[i] + 1.0 / 12.0 * c1[i];
    double dvel[3], Rq[9];
    oq q = oq_from_xyzw(s->q);
    if (cfg->iswithearth) {
        double cr[3], dvcg[3];
        v3_cross(cfg->iewn, s->v, cr);
        for (int i = 0; i < 3; i++) dvcg[i] = (cfg->gravity[i] - 2.0 * cr[i]) * dt;
        const double dnn[3] = {-cfg->iewn[0] * dt, -cfg->iewn[1] * dt, -cfg->iewn[2] * dt};
        const oq qnn = oq_from_rotvec(dnn);
        double Rnn[9], M1[9];
        oq_to_rot(qnn, Rnn);
        for (int i = 0; i < 9; i++) M1[i] = 0.5 * (((i % 4) == 0 ? 1.0 : 0.0) + Rnn[i]);
        oq_to_rot(q, Rq);
        m3m(M1, Rq, M1);
        m3v(M1, dvfb, dvel);
        for (int i = 0; i < 3; i++) dvel[i] = dvel[i] + dvcg[i];
        q = oq_normalized(oq_mul(oq_mul(qnn, q), oq_from_rotvec(dth)));
    } else {
        oq_to_rot(q, Rq);
        m3v(Rq, dvfb, dvel);
        for (int i = 0; i < 3; i++) dvel[i] = dvel[i] + cfg->gravity[i] * dt;
        q = oq_normalized(oq_mul(q, oq_from_rotvec(dth)));
    }
    oq_to_xyzw(q, s->q);
    for (int i = 0; i < 3; i++) s->p[i] += dt * s->v[i] + 0.5 * dt * dvel[i];
    for (int i = 0; i < 3; i++) s->v[i] += dvel[i];
}

void orc_ins_propagate(const orc_ins_config* cfg, const orc_imu* imu, int m, const orc_state* state0,
                       orc_state* states) {
    orc_state s = *state0;
    if (m > 0) states[0] = s;
    for (int k = 1; k < m; k++) {
        orc_ins_mechanization(cfg, &imu[k - 1], &imu[k], &s);
        states[k] = s;
    }
}

int orc_ins_window_index(const orc_imu* imu, int n, double t) {
    if (n == 0 || imu[0].time > t || imu[n - 1].time <= t) return 0;
    int sta = 0, end = n, counts = 0;
    for (;;) {
        const int mid = (sta + end) / 2;
        const double first = imu[mid - 1].time, second = imu[mid].time;
        if (first <= t && t < second) return mid;
        if (first > t)
            end = mid;
        else if (second <= t)
            sta = mid;
        if (counts++ > 15) return 0; /* the reference logs and returns index 0 */
    }
}

int orc_need_interpolation(const orc_imu* imu0, const orc_imu* imu1, double mid) {
    if (imu0->time < mid && imu1->time > mid) {
        if (mid - imu0->time < MIN_TIME_INTERVAL) return -1;
        if (imu1->time - mid < MIN_TIME_INTERVAL) return 1;
        return 2;
    }
    return 0;
}

void orc_imu_interpolation(const orc_imu* imu01, orc_imu* imu00, orc_imu* imu11, double mid) {
    const double scale = (imu01->time - mid) / imu01->dt;
    const orc_imu b = *imu01;
    imu00->time = mid;
    imu00->dt = b.dt - (b.time - mid);
    for (int i = 0; i < 3; i++) {
        imu00->dtheta[i] = b.dtheta[i] * (1 - scale);
        imu00->dvel[i] = b.dvel[i] * (1 - scale);
    }
    imu00->odovel = b.odovel * (1 - scale);
    imu11->time = b.time;
    imu11->dt = b.time - mid;
    for (int i = 0; i < 3; i++) {
        imu11->dtheta[i] = b.dtheta[i] * scale;
        imu11->dvel[i] = b.dvel[i] * scale;
    }
    imu11->odovel = b.odovel * scale;
}

int orc_redo_ins_mechanization(const orc_ins_config* cfg, const orc_state* updated, const orc_imu* imu, int n,
                               orc_state* states) {
    orc_state s = *updated;
    const int index = orc_ins_window_index(imu, n, s.time);
    if (index == 0) return 0;
    orc_imu imu0 = imu[index - 1], imu1 = imu[index];
    const int need = orc_need_interpolation(&imu0, &imu1, s.time);
    if (need == -1) {
        orc_ins_mechanization(cfg, &imu0, &imu1, &s);
        states[index] = s;
    } else if (need == 1) {
        s.time = imu1.time;
        states[index] = s;
    } else if (need == 2) {
        orc_imu_interpolation(&imu1, &imu0, &imu1, s.time);
        orc_ins_mechanization(cfg, &imu0, &imu1, &s);
        states[index] = s;
    }
    for (int k = index + 1; k < n; k++) {
        imu0 = imu1;
        imu1 = imu[k];
        orc_ins_mechanization(cfg, &imu0, &imu1, &s);
        states[k] = s;
    }
    return index;
}

int orc_imu_series_from_to(const orc_imu* imu, int n, double start, double end, orc_imu* series) {
    const int is = orc_ins_window_index(imu, n, start), ie = orc_ins_window_index(imu, n, end);
    /* the reference returns false only when both are 0; one 0 would read
       ins_windows[-1] there (out of range), so it is refused here too */
    if (is == 0 || ie == 0) return -1;
    int m = 0;
    orc_imu imu0 = imu[is - 1], imu1 = imu[is], tmp;
    int need = orc_need_interpolation(&imu0, &imu1, start);
    if (need == -1) {
        series[m++] = imu0;
        series[m++] = imu1;
    } else if (need == 1) {
        series[m++] = imu1;
    } else if (need == 2) {
        orc_imu_interpolation(&imu1, &tmp, &imu1, start);
        series[m++] = tmp;
        series[m++] = imu1;
    }
    for (int k = is + 1; k < ie - 1; k++) series[m++] = imu[k];
    imu0 = imu[ie - 1];
    imu1 = imu[ie];
    need = orc_need_interpolation(&imu0, &imu1, end);
    if (need == -1) {
        series[m++] = imu0;
    } else if (need == 1) {
        series[m++] = imu0;
        series[m++] = imu1;
    } else if (need == 2) {
        series[m++] = imu0;
        orc_imu_interpolation(&imu1, &tmp, &imu1, end);
        series[m++] = tmp;
    }
    if (m > 0) series[m - 1].time = end;
    return m;
}
