// api_ins.cpp -- C ABI of the INS mechanization and the IMU-series extraction
// (include/gvx.h): MISC::insMechanization / redoInsMechanization /
// getImuSeriesFromTo (/root/reference/ic_gvins/ic_gvins/misc.cc:40-384).  The
// window bookkeeping (binary search, interpolation split) is host logic, as in
// the reference; the mechanization chains run on the device (ins.hip).
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "gvx_internal.h"

using namespace gvx;

namespace {

constexpr double MIN_TIME_INTERVAL = 0.0001;  // MISC::MINIMUM_TIME_INTERVAL, misc.h:72

// MISC::getInsWindowIndex (misc.cc:40-83): first index with time > t, 0 = none.
int window_index(const gvx_imu* imu, int n, double t) {
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
        if (counts++ > 15) return 0;  // the reference logs and gives index 0
    }
}

// MISC::isNeedInterpolation (misc.cc:286-309)
int need_interpolation(const gvx_imu& imu0, const gvx_imu& imu1, double mid) {
    if (imu0.time < mid && imu1.time > mid) {
        if (mid - imu0.time < MIN_TIME_INTERVAL) return -1;
        if (imu1.time - mid < MIN_TIME_INTERVAL) return 1;
        return 2;
    }
    return 0;
}

// MISC::imuInterpolation (misc.cc:311-328); imu01 may alias imu11
void interpolate(const gvx_imu& imu01, gvx_imu& imu00, gvx_imu& imu11, double mid) {
    const double scale = (imu01.time - mid) / imu01.dt;
    const gvx_imu b = imu01;
    imu00.time = mid;
    imu00.dt = b.dt - (b.time - mid);
    for (int i = 0; i < 3; ++i) {
        imu00.dtheta[i] = b.dtheta[i] * (1 - scale);
        imu00.dvel[i] = b.dvel[i] * (1 - scale);
    }
    imu00.odovel = b.odovel * (1 - scale);
    imu11.time = b.time;
    imu11.dt = b.time - mid;
    for (int i = 0; i < 3; ++i) {
        imu11.dtheta[i] = b.dtheta[i] * scale;
        imu11.dvel[i] = b.dvel[i] * scale;
    }
    imu11.odovel = b.odovel * scale;
}

gvx_status check_cfg(gvx_ctx* c, const gvx_ins_config* cfg) {
    if (!cfg) return set_err(c, GVX_ERR_INVALID, "null INS configuration");
    return GVX_OK;
}

// Host chains -> device, run, copy every state back (synchronous).
gvx_status run_chains(gvx_ctx* c, const gvx_ins_config* cfg, int n_chain, const gvx_imu* imu, const int32_t* off,
                      const gvx_state* state0, gvx_state* states) {
    const size_t n_imu = (size_t)off[n_chain];
    // a pinned arena laid out like the device one: one upload of the inputs
    // (its prefix), one download of the states
    gvx_imu *d_imu, *h_imu;
    int32_t *d_off, *h_off;
    gvx_state *d_s0, *h_s0, *d_st, *h_st;
    Staging st;
    st.add(n_imu, &d_imu, &h_imu);
    st.add((size_t)n_chain + 1, &d_off, &h_off);
    st.add((size_t)n_chain, &d_s0, &h_s0);
    st.add(n_imu, &d_st, &h_st);
    void* db = scratch(c, "ins", st.bytes());
    void* hb = pinned(c, "ins", st.bytes());
    if (!db || !hb) return set_err(c, GVX_ERR_OOM, "INS staging");
    st.bind(db, hb);
    std::memcpy(h_imu, imu, n_imu * sizeof(gvx_imu));
    std::memcpy(h_off, off, sizeof(int32_t) * (n_chain + 1));
    std::memcpy(h_s0, state0, sizeof(gvx_state) * n_chain);
    hipError_t e = hipMemcpyAsync(d_imu, h_imu, (size_t)((char*)d_st - (char*)d_imu), hipMemcpyHostToDevice,
                                  c->stream);
    if (e != hipSuccess) return hip_err(c, e, "INS upload");
    hipEvent_t ev{};
    prof_begin(c, "ins", &ev);
    e = launch_ins(c, *cfg, n_chain, d_imu, d_off, d_s0, d_st);
    prof_end(c, "ins", ev);
    if (e != hipSuccess) return hip_err(c, e, "INS kernel");
    e = hipMemcpyAsync(h_st, d_st, sizeof(gvx_state) * n_imu, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "INS download");
    std::memcpy(states, h_st, sizeof(gvx_state) * n_imu);
    return GVX_OK;
}

}  // namespace

gvx_status gvx_ins_propagate_dev(gvx_ctx* c, const gvx_ins_config* cfg, int32_t n_chain, const gvx_imu* d_imu,
                                 const int32_t* d_off, const gvx_state* d_state0, gvx_state* d_states) {
    if (!c) return GVX_ERR_INVALID;
    gvx_status s = check_cfg(c, cfg);
    if (s) return s;
    if (n_chain < 0) return set_err(c, GVX_ERR_INVALID, "n_chain < 0");
    if (n_chain == 0) return GVX_OK;
    if (!d_imu || !d_off || !d_state0 || !d_states) return set_err(c, GVX_ERR_INVALID, "null device pointer");
    hipSetDevice(c->device);
    hipEvent_t ev{};
    prof_begin(c, "ins", &ev);
    hipError_t e = launch_ins(c, *cfg, n_chain, d_imu, d_off, d_state0, d_states);
    prof_end(c, "ins", ev);
    return hip_err(c, e, "INS kernel");
}

gvx_status gvx_ins_propagate(gvx_ctx* c, const gvx_ins_config* cfg, int32_t n_chain, const gvx_imu* imu,
                             const int32_t* off, const gvx_state* state0, gvx_state* states) {
    if (!c) return GVX_ERR_INVALID;
    gvx_status s = check_cfg(c, cfg);
    if (s) return s;
    if (n_chain < 0) return set_err(c, GVX_ERR_INVALID, "n_chain < 0");
    if (n_chain == 0) return GVX_OK;
    if (!imu || !off || !state0 || !states) return set_err(c, GVX_ERR_INVALID, "null pointer");
    if (off[0] != 0) return set_err(c, GVX_ERR_INVALID, "off[0] must be 0");
    for (int i = 0; i < n_chain; ++i)
        if (off[i + 1] < off[i]) return set_err(c, GVX_ERR_INVALID, "chain %d has negative length", i);
    hipSetDevice(c->device);
    return run_chains(c, cfg, n_chain, imu, off, state0, states);
}

gvx_status gvx_redo_ins_mechanization(gvx_ctx* c, const gvx_ins_config* cfg, const gvx_state* updated, int32_t n,
                                      const gvx_imu* imu, gvx_state* states, int32_t* index) {
    if (!c) return GVX_ERR_INVALID;
    gvx_status s = check_cfg(c, cfg);
    if (s) return s;
    if (!updated || !imu || !states || !index || n < 0) return set_err(c, GVX_ERR_INVALID, "bad INS window");
    *index = window_index(imu, n, updated->time);
    const int idx = *index;
    if (idx == 0) return GVX_OK;  // the reference logs "Failed to get right index" and returns
    gvx_imu imu0 = imu[idx - 1], imu1 = imu[idx];
    const int nd = need_interpolation(imu0, imu1, updated->time);
    // one chain: series[0] is the sample before the first mechanization step
    std::vector<gvx_imu> series;
    series.reserve((size_t)(n - idx + 2));
    gvx_state s0 = *updated;
    int first_out;  // window index of series[1]'s state
    if (nd == -1) {
        series.push_back(imu0);
        series.push_back(imu1);
        first_out = idx;
    } else if (nd == 1) {
        s0.time = imu1.time;
        states[idx] = s0;
        series.push_back(imu1);
        first_out = idx + 1;
    } else if (nd == 2) {
        interpolate(imu1, imu0, imu1, updated->time);
        series.push_back(imu0);
        series.push_back(imu1);
        first_out = idx;
    } else {
        series.push_back(imu1);  // state unchanged at idx; the loop starts from window[idx]
        first_out = idx + 1;
    }
    for (int k = idx + 1; k < n; ++k) series.push_back(imu[k]);
    const int m = (int)series.size();
    if (m < 2) return GVX_OK;
    hipSetDevice(c->device);
    std::vector<gvx_state> out((size_t)m);
    const int32_t off[2] = {0, m};
    s = run_chains(c, cfg, 1, series.data(), off, &s0, out.data());
    if (s) return s;
    std::memcpy(states + first_out, out.data() + 1, sizeof(gvx_state) * (size_t)(m - 1));
    return GVX_OK;
}

gvx_status gvx_imu_series_from_to(const gvx_imu* imu, int32_t n, double start, double end, gvx_imu* series,
                                  int32_t* n_series) {
    if (!imu || !series || !n_series || n < 0) return GVX_ERR_INVALID;
    const int is = window_index(imu, n, start), ie = window_index(imu, n, end);
    *n_series = 0;
    // the reference fails only when both are 0; one 0 would index window[-1] there
    if (is == 0 || ie == 0) return GVX_ERR_NOT_FOUND;
    int m = 0;
    gvx_imu imu0 = imu[is - 1], imu1 = imu[is], tmp{};
    int nd = need_interpolation(imu0, imu1, start);
    if (nd == -1) {
        series[m++] = imu0;
        series[m++] = imu1;
    } else if (nd == 1) {
        series[m++] = imu1;
    } else if (nd == 2) {
        interpolate(imu1, tmp, imu1, start);
        series[m++] = tmp;
        series[m++] = imu1;
    }
    for (int k = is + 1; k < ie - 1; ++k) series[m++] = imu[k];
    imu0 = imu[ie - 1];
    imu1 = imu[ie];
    nd = need_interpolation(imu0, imu1, end);
    if (nd == -1) {
        series[m++] = imu0;
    } else if (nd == 1) {
        series[m++] = imu0;
        series[m++] = imu1;
    } else if (nd == 2) {
        series[m++] = imu0;
        interpolate(imu1, tmp, imu1, end);
        series[m++] = tmp;
    }
    if (m > 0) series[m - 1].time = end;
    *n_series = m;
    return GVX_OK;
}
